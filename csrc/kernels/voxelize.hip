// K7 — deterministic point -> voxel assignment with spconv VoxelGenerator
// semantics (reference: clients/preprocess/preprocess_3d.py:46-50 via OpenPCDet
// transform_points_to_voxels / spconv; clients/preprocess/voxelize.py:40-47 via det3d).
//
// spconv semantics reproduced exactly (bit-for-bit voxel ids and slot order):
//  * points outside the range (floor((p - min) / size) outside the grid) are dropped;
//  * voxel ids are assigned in order of each voxel's FIRST point index;
//    voxels whose first point comes after max_voxels voxels exist are dropped
//    (spconv 2.x `continue` semantics);
//  * a voxel keeps its first `max_points` points in point order.
//
// Parallel scheme (5 launches, batched over B frames, no host sync):
//  a) per point: cell id, atomicMin(cell_first[cell], i)
//  b1) per 1024-point block: count points that are their cell's first point
//  b2) per block: ordered prefix -> voxel id of each first point (< max_voxels),
//      cell_vid[cell] = vid, coords[vid] = (b, z, y, x), voxel_count
//  c) per point: vid = cell_vid[cell]; count[vid]++; insert i into the voxel's
//      sorted slot list with the atomicMin carry chain (values in a slot only
//      ever decrease, so slot k converges to the k-th smallest index; a
//      non-atomic read lets a thread skip slots that already hold a smaller
//      index) -> the first max_points indices, in order, independent of timing
//  d) per voxel (one wave): gather features into voxels[V][P][F] (optional —
//      the fused PointPillars path gathers inside its VFE kernel instead),
//      num_points = min(count, P); reset the voxel's slots; plus per point:
//      reset cell_first / cell_vid.
// All scratch is self-resetting, so the dense cell grids (even the 90 M-cell
// SECOND grid: 720 MB, affordable in 288 GB of HBM) are cleared in O(points)
// per frame instead of O(cells); they are initialised once at allocation.
#include <cstdlib>

#include "tca_common.h"

using namespace tca;

namespace {

constexpr int kBlock = 256;
constexpr int kPPT = 4;  // points per thread in the scan kernels
constexpr int kPtsPerBlock = kBlock * kPPT;
constexpr int kEmpty = 0x7fffffff;

struct VoxGeom {
  float r0, r1, r2;      // range min
  float vs0, vs1, vs2;   // voxel size
  int nx, ny, nz;
  long cells;            // per-frame rows of cell_first / cell_vid: nx*ny*nz (dense) or the hash table size
  int* keys;             // hash mode: per-frame open-addressing table [B][cells] of cell ids (-1 empty), else null
  int hbits;             // log2 of the hash table size
};

// Hash mode (grids far larger than a frame's points, e.g. SECOND's 1408 x 1600 x 40): a cell's
// row is its slot in a per-frame linear-probing table of >= 2x max_points entries (load <= 1/2),
// claimed by atomicCAS on the key; point_cell then holds the slot, every later stage indexes
// by it unchanged, and the cell id (for coords) is read back from the key.  Voxel ids depend
// only on each cell's first point index, so the results equal the dense grid's bit for bit.
__device__ __forceinline__ int hash_slot(int* keys, int hbits, int cell) {
  const unsigned mask = (1u << hbits) - 1u;
  unsigned h = ((unsigned)cell * 0x9E3779B1u) >> (32 - hbits);
  while (true) {
    const int k = atomicCAS(&keys[h], -1, cell);
    if (k == -1 || k == cell) return (int)h;
    h = (h + 1u) & mask;
  }
}

template <bool NT = false>
__device__ __forceinline__ int cell_of(const float* p, const VoxGeom& g, int& cx, int& cy, int& cz) {
  const float x = NT ? __builtin_nontemporal_load(p) : p[0];
  const float y = NT ? __builtin_nontemporal_load(p + 1) : p[1];
  const float z = NT ? __builtin_nontemporal_load(p + 2) : p[2];
  cx = (int)floorf((x - g.r0) / g.vs0);
  cy = (int)floorf((y - g.r1) / g.vs1);
  cz = (int)floorf((z - g.r2) / g.vs2);
  if (cx < 0 || cx >= g.nx || cy < 0 || cy >= g.ny || cz < 0 || cz >= g.nz) return -1;
  return (cz * g.ny + cy) * g.nx + cx;
}

// Runs of equal keys in consecutive lanes.  A sensor's points arrive ring by ring in azimuth
// order, so neighbouring points mostly fall into the same pillar (at 10 m, ~5 consecutive points of
// a 1875-step ring share a 16 cm pillar): one atomic per run instead of one per point.  key < 0:
// no key (never part of a run).  head: the run's first lane (the smallest point index of the run);
// len: the run's length (valid on the head); rank / head_lane: this lane's place in its run.
struct Run {
  bool head;
  int len, rank, head_lane;
};

__device__ __forceinline__ Run wave_run(int key) {
  const int lane = threadIdx.x & 63;
  const int prev = __shfl_up(key, 1, 64);
  Run r;
  r.head = key >= 0 && (lane == 0 || prev != key);
  const unsigned long long brk = __ballot(key < 0 || r.head);  // every run starts at a break
  const unsigned long long after = lane == 63 ? 0ull : (brk >> (lane + 1));
  r.len = after ? (__builtin_ctzll(after) + 1) : (64 - lane);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  r.head_lane = 63 - __builtin_clzll(brk & upto);  // lane's own break or the last one before it
  r.rank = lane - r.head_lane;
  return r;
}

// NT (TCA_VOX_NT=1): the point coordinates (vox_cell) and point_cell's last read (vox_cell_reset) as
// non-temporal loads
template <bool NT>
__global__ void __launch_bounds__(kBlock) vox_cell_kernel(const float* __restrict__ pts, int pstride, int max_pts,
                                                          const int* __restrict__ npts, VoxGeom g,
                                                          int* __restrict__ cell_first, int* __restrict__ point_cell) {
  const int b = blockIdx.y, n = npts[b];
  for (int ch = blockIdx.x; ch * kBlock < max_pts; ch += gridDim.x) {  // 256-point chunks (vox_pgrid)
    const int i = ch * kBlock + threadIdx.x;
    int cell = -1;
    if (i < max_pts && i < n) {
      const float* p = pts + ((long)b * max_pts + i) * pstride;
      int cx, cy, cz;
      cell = cell_of<NT>(p, g, cx, cy, cz);
    }
    // the run head holds the run's smallest index: atomicMin of the others cannot change the cell
    const Run r = wave_run(cell);
    if (g.keys) {  // hash mode: the head claims the run's table slot
      int slot = r.head ? hash_slot(g.keys + (long)b * g.cells, g.hbits, cell) : -1;
      slot = __shfl(slot, r.head_lane, 64);
      if (cell >= 0) cell = slot;
    }
    if (r.head) atomicMin(&cell_first[(long)b * g.cells + cell], i);
    if (i < max_pts) point_cell[(long)b * max_pts + i] = cell;
  }
}

__device__ __forceinline__ int first_flag(const int* pc, const int* cf, long cbase, int i, int n) {
  if (i >= n) return 0;
  const int c = pc[i];
  return (c >= 0 && cf[cbase + c] == i) ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock) vox_count_first_kernel(const int* __restrict__ point_cell, int max_pts,
                                                                 const int* __restrict__ npts, long cells,
                                                                 const int* __restrict__ cell_first, int bpf,
                                                                 int* __restrict__ block_count) {
  __shared__ int s[kBlock / 64];
  const int b = blockIdx.y, blk = blockIdx.x;
  const int n = npts[b];
  const int* pc = point_cell + (long)b * max_pts;
  const long cbase = (long)b * cells;
  int cnt = 0;
  const int first = blk * kPtsPerBlock + threadIdx.x * kPPT;
#pragma unroll
  for (int k = 0; k < kPPT; ++k) cnt += first_flag(pc, cell_first, cbase, first + k, n);
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
    for (int k = 0; k < kBlock / 64; ++k) c += s[k];
    block_count[b * bpf + blk] = c;
  }
}

__global__ void __launch_bounds__(kBlock) vox_assign_kernel(const int* __restrict__ point_cell, int max_pts,
                                                            const int* __restrict__ npts, VoxGeom g,
                                                            const int* __restrict__ cell_first, int bpf,
                                                            const int* __restrict__ block_count, int max_voxels,
                                                            int* __restrict__ cell_vid, int* __restrict__ coords,
                                                            int* __restrict__ voxel_count) {
  __shared__ int s_scan[kBlock / 64 + 1];
  __shared__ int s_prefix;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int n = npts[b];
  const int* pc = point_cell + (long)b * max_pts;
  const long cbase = (long)b * g.cells;
  if (threadIdx.x < 64) {
    int acc = 0;
    for (int k = threadIdx.x; k < blk; k += 64) acc += block_count[b * bpf + k];
    acc = wave_sum(acc);
    if (threadIdx.x == 0) s_prefix = acc;
    if (blk == bpf - 1) {
      int tot = 0;
      for (int k = threadIdx.x; k < bpf; k += 64) tot += block_count[b * bpf + k];
      tot = wave_sum(tot);
      if (threadIdx.x == 0) voxel_count[b] = min(tot, max_voxels);
    }
  }
  int f[kPPT];
  int cnt = 0;
  const int first = blk * kPtsPerBlock + threadIdx.x * kPPT;
#pragma unroll
  for (int k = 0; k < kPPT; ++k) { f[k] = first_flag(pc, cell_first, cbase, first + k, n); cnt += f[k]; }
  int total;
  int vid = block_excl_scan(cnt, s_scan, &total) + s_prefix;
#pragma unroll
  for (int k = 0; k < kPPT; ++k) {
    if (!f[k]) continue;
    if (vid < max_voxels) {
      const int c = pc[first + k];
      cell_vid[cbase + c] = vid;
      const int cell = g.keys ? g.keys[cbase + c] : c;
      const int cx = cell % g.nx, cy = (cell / g.nx) % g.ny, cz = cell / (g.nx * g.ny);
      int* co = coords + ((long)b * max_voxels + vid) * 4;
      co[0] = b; co[1] = cz; co[2] = cy; co[3] = cx;
    }
    ++vid;
  }
}

__global__ void __launch_bounds__(kBlock) vox_insert_kernel(const int* __restrict__ point_cell, int max_pts,
                                                            const int* __restrict__ npts, long cells,
                                                            const int* __restrict__ cell_vid, int max_voxels, int P,
                                                            int* __restrict__ vcount, int* __restrict__ slots) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npts[b] || i >= max_pts) return;
  const int c = point_cell[(long)b * max_pts + i];
  if (c < 0) return;
  const int vid = cell_vid[(long)b * cells + c];
  if (vid < 0) return;
  const long v = (long)b * max_voxels + vid;
  atomicAdd(&vcount[v], 1);
  int* s = slots + v * P;
  int val = i;
  // Slot values only ever decrease and the list stays sorted, so a slot seen
  // holding a smaller index holds one forever: binary-search the first slot
  // not yet known to be smaller (log2 P dependent loads instead of a walk of
  // up to P), and leave at once when even the last slot is smaller (the point
  // is not among its voxel's first P).
  int lo = 0, hi = P;  // invariant: s[0 .. lo) < val was observed
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (__hip_atomic_load(&s[mid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < val) lo = mid + 1;
    else hi = mid;
  }
  for (int k = lo; k < P; ++k) {
    const int cur = __hip_atomic_load(&s[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur < val) continue;  // slot already (permanently) holds a smaller index
    const int old = atomicMin(&s[k], val);
    if (old == kEmpty) return;
    if (old > val) val = old;  // displaced a larger index: carry it on
  }
}

// Grid-stride, bounded grid (dispatching B*V early-exit blocks would cost
// more than the work): each wave walks voxels (gather + slot reset), then the
// whole grid walks points (cell-grid reset).
__global__ void __launch_bounds__(256) vox_gather_reset_kernel(
    const float* __restrict__ pts, int pstride, int max_pts, const int* __restrict__ npts, int nfeat, int batch,
    int max_voxels, int P, const int* __restrict__ voxel_count, int* __restrict__ vcount, int* __restrict__ slots,
    float* __restrict__ voxels, int* __restrict__ num_points, const int* __restrict__ point_cell, long cells,
    int* __restrict__ cell_first, int* __restrict__ cell_vid, int* __restrict__ keys, int gather) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  const long nv = (long)batch * max_voxels;
  for (long g = wave; g < nv; g += nwaves) {
    const int b = (int)(g / max_voxels), vid = (int)(g - (long)b * max_voxels);
    if (vid >= voxel_count[b]) {  // skip the rest of this frame's empty tail
      continue;
    }
    const int cnt = vcount[g];
    const int n = min(cnt, P);
    int* s = slots + g * P;
    for (int k = lane; k < P; k += 64) {
      const int idx = s[k];
      if (gather) {
        float* o = voxels + (g * P + k) * nfeat;
        if (k < n) {
          const float* p = pts + ((long)b * max_pts + idx) * pstride;
          for (int f = 0; f < nfeat; ++f) o[f] = p[f];
        } else {
          for (int f = 0; f < nfeat; ++f) o[f] = 0.f;
        }
      }
      s[k] = kEmpty;  // each lane resets only the slots it read itself
    }
    if (lane == 0) { num_points[g] = n; vcount[g] = 0; }
  }
  const long np = (long)batch * max_pts;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < np; t += (long)gridDim.x * blockDim.x) {
    const int b = (int)(t / max_pts), i = (int)(t - (long)b * max_pts);
    if (i >= npts[b]) continue;
    const int c = point_cell[t];
    if (c < 0) continue;
    cell_first[(long)b * cells + c] = kEmpty;
    cell_vid[(long)b * cells + c] = -1;
    if (keys) keys[(long)b * cells + c] = -1;
  }
}

// ---- stage c, CSR form -------------------------------------------------------
// Sorted first-P slot lists without the atomicMin carry chain.  The chain
// makes each point walk its voxel's slots with dependent device-scope atomics
// (resolved at the memory side on this part, ~1-2 us each), so one dense
// pillar's chain sets the kernel time.  Instead, a counting sort:
//  c1) per point: vcount[vid]++ (no-return atomic)
//  c2) per frame: exclusive scan of vcount -> offs, cursor = offs
//  c3) per point: csr[atomicAdd(cursor[vid], 1)] = i (one round trip)
//  c4) per voxel: count <= 8 (~95% of pillars) -> 8-wide sorting network in
//      registers; denser voxels are listed and
//  c5) one wave per dense voxel keeps the smallest min(count, P) indices by
//      64-lane bitonic sort + merge over 64-index chunks.
__global__ void __launch_bounds__(kBlock) vox_count_kernel(const int* __restrict__ point_cell, int max_pts,
                                                           const int* __restrict__ npts, long cells,
                                                           const int* __restrict__ cell_vid, int max_voxels,
                                                           int* __restrict__ vcount) {
  const int b = blockIdx.y, n = npts[b];
  for (int ch = blockIdx.x; ch * kBlock < max_pts; ch += gridDim.x) {  // 256-point chunks (vox_pgrid)
    const int i = ch * kBlock + threadIdx.x;
    int vid = -1;
    if (i < n && i < max_pts) {
      const int c = point_cell[(long)b * max_pts + i];
      if (c >= 0) vid = cell_vid[(long)b * cells + c];
    }
    const Run r = wave_run(vid);  // one atomic per run of points in one voxel
    if (r.head) atomicAdd(&vcount[(long)b * max_voxels + vid], r.len);
  }
}

constexpr int kScanT = 1024;

__global__ void __launch_bounds__(kScanT) vox_scan_kernel(const int* __restrict__ voxel_count, int max_voxels,
                                                          const int* __restrict__ vcount, int* __restrict__ offs,
                                                          int* __restrict__ cursor, int* __restrict__ dense_count) {
  // chunks of kScanT counts, one per thread, read and written coalesced; a block scan per chunk
  __shared__ int s_w[kScanT / 64];
  __shared__ int s_carry;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int n = voxel_count[b];
  const int* vc = vcount + (long)b * max_voxels;
  int* ob = offs + (long)b * (max_voxels + 1);
  int* cb = cursor + (long)b * max_voxels;
  if (t == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += kScanT) {
    const int v = base + t;
    const int x = v < n ? vc[v] : 0;
    const int incl = wave_incl_sum(x);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    int wbase = s_carry;
    for (int w = 0; w < wid; ++w) wbase += s_w[w];
    const int excl = wbase + incl - x;
    if (v < n) {
      ob[v] = excl;
      cb[v] = excl;
    }
    __syncthreads();  // every thread has read s_w and s_carry
    if (t == kScanT - 1) s_carry = excl + x;
    __syncthreads();
  }
  if (t == 0) {
    ob[n] = s_carry;
    dense_count[b] = 0;
  }
}

__global__ void __launch_bounds__(kBlock) vox_fill_kernel(const int* __restrict__ point_cell, int max_pts,
                                                          const int* __restrict__ npts, long cells,
                                                          const int* __restrict__ cell_vid, int max_voxels,
                                                          int* __restrict__ cursor, int* __restrict__ csr) {
  const int b = blockIdx.y, n = npts[b];
  for (int ch = blockIdx.x; ch * kBlock < max_pts; ch += gridDim.x) {  // 256-point chunks (vox_pgrid)
    const int i = ch * kBlock + threadIdx.x;
    int vid = -1;
    if (i < n && i < max_pts) {
      const int c = point_cell[(long)b * max_pts + i];
      if (c >= 0) vid = cell_vid[(long)b * cells + c];
    }
    // one cursor atomic per run: the head reserves the run's positions, its lanes take them in order
    // (a voxel's list is sorted by the next stage, so only the set of positions matters)
    const Run r = wave_run(vid);
    int base = 0;
    if (r.head) base = atomicAdd(&cursor[(long)b * max_voxels + vid], r.len);
    base = __shfl(base, r.head_lane, 64);
    if (vid >= 0) csr[(long)b * max_pts + base + r.rank] = i;
  }
}

__device__ __forceinline__ void cswap(int& a, int& b) {
  const int lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}

__global__ void __launch_bounds__(kBlock) vox_sort_small_kernel(int max_voxels, int max_pts, int P,
                                                                const int* __restrict__ voxel_count,
                                                                const int* __restrict__ vcount,
                                                                const int* __restrict__ offs,
                                                                const int* __restrict__ csr, int* __restrict__ slots,
                                                                int* __restrict__ dense, int* __restrict__ dense_count) {
  const int b = blockIdx.y, vid = blockIdx.x * blockDim.x + threadIdx.x;
  if (vid >= voxel_count[b]) return;
  const long g = (long)b * max_voxels + vid;
  const int c = vcount[g];
  if (c > 8) {
    dense[(long)b * max_voxels + atomicAdd(&dense_count[b], 1)] = vid;
    return;
  }
  const int* src = csr + (long)b * max_pts + offs[(long)b * (max_voxels + 1) + vid];
  int a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = k < c ? src[k] : kEmpty;
  // Batcher odd-even merge sort, 19 comparators (static indices: registers only)
  cswap(a[0], a[1]); cswap(a[2], a[3]); cswap(a[4], a[5]); cswap(a[6], a[7]);
  cswap(a[0], a[2]); cswap(a[1], a[3]); cswap(a[4], a[6]); cswap(a[5], a[7]);
  cswap(a[1], a[2]); cswap(a[5], a[6]); cswap(a[0], a[4]); cswap(a[3], a[7]);
  cswap(a[1], a[5]); cswap(a[2], a[6]); cswap(a[1], a[4]); cswap(a[3], a[6]);
  cswap(a[2], a[4]); cswap(a[3], a[5]); cswap(a[3], a[4]);
  int* s = slots + g * P;
  const int m = min(c, P);
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < m) s[k] = a[k];
}

__device__ __forceinline__ int bitonic_sort64(int v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = __shfl_xor(v, j, 64);
      const bool up = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == up) ? min(v, o) : max(v, o);
    }
  return v;
}

__global__ void __launch_bounds__(256) vox_sort_dense_kernel(int max_voxels, int max_pts, int P,
                                                             const int* __restrict__ vcount,
                                                             const int* __restrict__ offs,
                                                             const int* __restrict__ csr, const int* __restrict__ dense,
                                                             const int* __restrict__ dense_count,
                                                             int* __restrict__ slots) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nd = dense_count[b];
  for (int d = wave; d < nd; d += nwaves) {
    const int vid = dense[(long)b * max_voxels + d];
    const long g = (long)b * max_voxels + vid;
    const int c = vcount[g];
    const int* src = csr + (long)b * max_pts + offs[(long)b * (max_voxels + 1) + vid];
    int best = kEmpty;  // ascending across lanes: the 64 smallest so far
    for (int base = 0; base < c; base += 64) {
      int v = base + lane < c ? src[base + lane] : kEmpty;
      v = bitonic_sort64(v, lane);
      // smallest 64 of two ascending runs: min(best[l], v[63 - l]) is bitonic; clean it
      int m = min(best, __shfl(v, 63 - lane, 64));
#pragma unroll
      for (int j = 32; j > 0; j >>= 1) {
        const int o = __shfl_xor(m, j, 64);
        m = (lane & j) == 0 ? min(m, o) : max(m, o);
      }
      best = m;
    }
    if (lane < min(c, P)) slots[g * P + lane] = best;
  }
}

// Reset pass of the fused path (no gather), split for memory-level
// parallelism: one thread per 16-B chunk of a voxel's slot row (P % 4 == 0)
// instead of a wave per voxel writing 4-B slots, and one thread per point for
// the cell tables.
__global__ void __launch_bounds__(256) vox_slot_reset_kernel(int max_voxels, int P, const int* __restrict__ voxel_count,
                                                             int* __restrict__ vcount, int* __restrict__ slots,
                                                             int* __restrict__ num_points) {
  const int b = blockIdx.y;
  const int cpv = P >> 2;  // 16-B chunks per voxel
  const int n = voxel_count[b] * cpv;
  const bool pow2 = (cpv & (cpv - 1)) == 0;
  const int sh = __builtin_ctz(cpv);
  for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {  // bounded grid
    const int vid = pow2 ? t >> sh : t / cpv, c = t - vid * cpv;
    const long g = (long)b * max_voxels + vid;
    reinterpret_cast<int4*>(slots + g * P)[c] = make_int4(kEmpty, kEmpty, kEmpty, kEmpty);
    if (c == 0) {
      num_points[g] = min(vcount[g], P);
      vcount[g] = 0;
    }
  }
}

template <bool NT>
__global__ void __launch_bounds__(256) vox_cell_reset_kernel(int max_pts, const int* __restrict__ npts,
                                                             const int* __restrict__ point_cell, long cells,
                                                             int* __restrict__ cell_first, int* __restrict__ cell_vid,
                                                             int* __restrict__ keys) {
  const int b = blockIdx.y, n = npts[b];
  for (int ch = blockIdx.x; ch * 256 < max_pts; ch += gridDim.x) {  // 256-point chunks (vox_pgrid)
    const int i = ch * 256 + threadIdx.x;
    const int* pc = point_cell + (long)b * max_pts + i;
    const int c = i < n && i < max_pts ? (NT ? __builtin_nontemporal_load(pc) : *pc) : -1;
    if (!wave_run(c).head) continue;  // one reset per run of points in one cell
    cell_first[(long)b * cells + c] = kEmpty;
    cell_vid[(long)b * cells + c] = -1;
    if (keys) keys[(long)b * cells + c] = -1;
  }
}

// workgroups per frame of the per-point passes (vox_cell / vox_count / vox_fill / vox_cell_reset): each
// walks 256-point chunks blockIdx.x, blockIdx.x + gridDim.x, ... .  One chunk per workgroup (15,104
// workgroups per 32-sweep batch) floods the dispatcher beside the BEV convs; TCA_VOX_GRID caps it
int vox_pgrid(int max_points) {
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("TCA_VOX_GRID");
    cap = e ? atoi(e) : 0;
    cap = cap < 0 ? 0 : cap;
  }
  const int chunks = (max_points + kBlock - 1) / kBlock;
  return cap > 0 && cap < chunks ? cap : chunks;
}

bool vox_nt() {
  static const bool nt = getenv("TCA_VOX_NT") && atoi(getenv("TCA_VOX_NT")) != 0;
  return nt;
}

VoxGeom make_geom(const float* range, const float* vsize, const int* grid, int* keys, int hbits) {
  VoxGeom g;
  g.r0 = range[0]; g.r1 = range[1]; g.r2 = range[2];
  g.vs0 = vsize[0]; g.vs1 = vsize[1]; g.vs2 = vsize[2];
  g.nx = grid[0]; g.ny = grid[1]; g.nz = grid[2];
  g.keys = hbits > 0 ? keys : nullptr;
  g.hbits = hbits;
  g.cells = g.keys ? (1L << hbits) : (long)g.nx * g.ny * g.nz;
  return g;
}

}  // namespace

TCA_API int tca_vox_blocks_per_frame(int max_points) { return (max_points + kPtsPerBlock - 1) / kPtsPerBlock; }

// Scratch contract (allocated once, initialised once, self-resetting):
//   cell_first int[B*cells] = INT_MAX, cell_vid int[B*cells] = -1,
//   slots int[B*V*P] = INT_MAX, vcount int[B*V] = 0,
//   point_cell int[B*max_points], block_count int[B*blocks_per_frame].
// Hash mode (hash_bits > 0): cell_first / cell_vid / keys are int[B << hash_bits] (keys = -1) with
// 1 << hash_bits >= 2 * max_points; dense (hash_bits = 0, keys unused): int[B*cells].
// Stages: mode bit 1 = run assignment (a,b1,b2,c); bit 2 = run gather/reset (d).
// The fused PointPillars path runs mode 1, then its VFE kernel consumes the
// slots, then mode 2 with gather = 0 to reset.
TCA_API int tca_voxelize(const float* pts, int pstride, int max_points, const int* npts, int batch,
                         const float* range, const float* vsize, const int* grid, int P, int max_voxels, int nfeat,
                         int* cell_first, int* cell_vid, int* point_cell, int* block_count, int* slots, int* vcount,
                         float* voxels, int* coords, int* num_points, int* voxel_count, int mode, int gather,
                         int* keys, int hash_bits, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (hash_bits < 0 || hash_bits > 30 || (hash_bits > 0 && (!keys || (1L << hash_bits) < 2L * max_points)))
    return (int)hipErrorInvalidValue;  // the probe loop needs free slots: load <= 1/2
  VoxGeom g = make_geom(range, vsize, grid, keys, hash_bits);
  const int bpf = (max_points + kPtsPerBlock - 1) / kPtsPerBlock;
  dim3 pgrid(vox_pgrid(max_points), batch);
  dim3 sgrid(bpf, batch);
  if (mode & 1) {
    (vox_nt() ? vox_cell_kernel<true> : vox_cell_kernel<false>)<<<pgrid, kBlock, 0, stream>>>(pts, pstride, max_points, npts, g, cell_first, point_cell);
    vox_count_first_kernel<<<sgrid, kBlock, 0, stream>>>(point_cell, max_points, npts, g.cells, cell_first, bpf,
                                                         block_count);
    vox_assign_kernel<<<sgrid, kBlock, 0, stream>>>(point_cell, max_points, npts, g, cell_first, bpf, block_count,
                                                    max_voxels, cell_vid, coords, voxel_count);
    if (!(mode & 4))
      vox_insert_kernel<<<pgrid, kBlock, 0, stream>>>(point_cell, max_points, npts, g.cells, cell_vid, max_voxels, P,
                                                      vcount, slots);
  }
  if ((mode & 2) && !gather && (P & 3) == 0) {
    const int need = (max_voxels * (P / 4) + 255) / 256;
    vox_slot_reset_kernel<<<dim3(need < 32 ? need : 32, batch), 256, 0, stream>>>(
        max_voxels, P, voxel_count, vcount, slots, num_points);
    (vox_nt() ? vox_cell_reset_kernel<true> : vox_cell_reset_kernel<false>)<<<pgrid, kBlock, 0, stream>>>(max_points, npts, point_cell, g.cells, cell_first, cell_vid,
                                                        g.keys);
  } else if (mode & 2) {
    vox_gather_reset_kernel<<<1024, 256, 0, stream>>>(pts, pstride, max_points, npts, nfeat, batch,
                                                               max_voxels, P, voxel_count, vcount, slots, voxels,
                                                               num_points, point_cell, g.cells, cell_first, cell_vid,
                                                               g.keys, gather);
  }
  TCA_LAUNCH_CHECK();
}

// Stage c in CSR form (see vox_count_kernel): run after tca_voxelize(mode 1 | 4).
// Scratch: offs int[B*(V+1)], cursor int[B*V], csr int[B*max_points],
// dense int[B*V], dense_count int[B].  Requires P <= 64.
TCA_API int tca_vox_slots_csr(const int* point_cell, int max_points, const int* npts, int batch, const int* grid,
                              const int* cell_vid, int max_voxels, int P, const int* voxel_count, int* vcount,
                              int* offs, int* cursor, int* csr, int* dense, int* dense_count, int* slots,
                              int hash_bits, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (P > 64 || P < 1) return (int)hipErrorInvalidValue;
  const long cells = hash_bits > 0 ? (1L << hash_bits) : (long)grid[0] * grid[1] * grid[2];
  dim3 pgrid(vox_pgrid(max_points), batch);
  vox_count_kernel<<<pgrid, kBlock, 0, stream>>>(point_cell, max_points, npts, cells, cell_vid, max_voxels, vcount);
  vox_scan_kernel<<<batch, kScanT, 0, stream>>>(voxel_count, max_voxels, vcount, offs, cursor, dense_count);
  vox_fill_kernel<<<pgrid, kBlock, 0, stream>>>(point_cell, max_points, npts, cells, cell_vid, max_voxels, cursor,
                                                csr);
  vox_sort_small_kernel<<<dim3((max_voxels + kBlock - 1) / kBlock, batch), kBlock, 0, stream>>>(
      max_voxels, max_points, P, voxel_count, vcount, offs, csr, slots, dense, dense_count);
  vox_sort_dense_kernel<<<dim3(64, batch), 256, 0, stream>>>(max_voxels, max_points, P, vcount, offs, csr, dense,
                                                             dense_count, slots);
  TCA_LAUNCH_CHECK();
}
