// Sanitizer driver for csrc/runtime/rccl_comm.cpp's plan building and argument
// checks.  Built host-only with the stand-in headers under rccl_stub/ (no GPU,
// no librccl): the RCCL entry points below record every call and touch every
// byte a real transfer would (read a send buffer, write a recv buffer) over the
// element count the wrapper computed, so ASan reports any count / dtype error as
// an overflow of the exactly-sized heap buffer.  Random plans (valid and not)
// are checked against the expected op list; an invalid plan must post nothing.
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct ncclComm {
  int nranks;
  int rank;
};

namespace {
struct Op {
  int kind;  // 0 send, 1 recv, 2 allreduce, 3 broadcast
  const void* buf;
  size_t count;
  ncclDataType_t dt;
  int peer;
};
std::vector<Op> g_ops;
int g_depth = 0, g_groups = 0;
unsigned char g_sink = 0;

size_t esize(ncclDataType_t dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

void touch_read(const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) g_sink ^= b[i];
}

int fail(const char* what, int it) {
  std::fprintf(stderr, "rccl plan fuzz: %s (iteration %d)\n", what, it);
  return 1;
}
}  // namespace

extern "C" {
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id, 7, sizeof(*id));
  return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
  *comm = new ncclComm{nranks, rank};
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t comm) { return ncclCommDestroy(comm); }
ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t* err) {
  *err = ncclSuccess;
  return ncclSuccess;
}
ncclResult_t ncclCommCount(ncclComm_t comm, int* count) {
  *count = comm->nranks;
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "stub"; }
ncclResult_t ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  --g_depth;
  ++g_groups;
  return ncclSuccess;
}
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  if (g_depth <= 0 || peer < 0 || peer >= comm->nranks) return ncclInvalidUsage;
  touch_read(buf, count * esize(dt));
  g_ops.push_back({0, buf, count, dt, peer});
  return ncclSuccess;
}
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  if (g_depth <= 0 || peer < 0 || peer >= comm->nranks) return ncclInvalidUsage;
  std::memset(buf, 0x5a, count * esize(dt));
  g_ops.push_back({1, buf, count, dt, peer});
  return ncclSuccess;
}
ncclResult_t ncclAllReduce(const void* sb, void* rb, size_t count, ncclDataType_t dt, ncclRedOp_t, ncclComm_t,
                           hipStream_t) {
  touch_read(sb, count * esize(dt));
  if (count) std::memset(rb, 0, count * esize(dt));
  g_ops.push_back({2, rb, count, dt, -1});
  return ncclSuccess;
}
ncclResult_t ncclBroadcast(const void* sb, void* rb, size_t count, ncclDataType_t dt, int root, ncclComm_t comm,
                           hipStream_t) {
  if (root < 0 || root >= comm->nranks) return ncclInvalidUsage;
  touch_read(sb, count * esize(dt));
  if (count) std::memset(rb, 1, count * esize(dt));
  g_ops.push_back({3, rb, count, dt, root});
  return ncclSuccess;
}

// the wrappers under test (csrc/runtime/rccl_comm.cpp)
int tca_rccl_unique_id_bytes();
int tca_rccl_get_unique_id(void* out);
int tca_rccl_comm_init(void** comm_out, int nranks, const void* id_bytes, int rank);
int tca_rccl_comm_destroy(void* comm);
int tca_rccl_async_error(void* comm);
int tca_rccl_comm_count(void* comm, int* count);
int tca_rccl_group_p2p(void* comm, int n, const int* kind, const int* peer, void* const* buf, const int64_t* bytes,
                       void* stream);
int tca_rccl_allreduce_max_f64(void* comm, double* buf, int64_t n, void* stream);
int tca_rccl_broadcast(void* comm, void* buf, int64_t nbytes, int root, void* stream);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  std::mt19937 rng(12345);
  auto pick = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
  const int64_t sizes[] = {-3, 0, 1, 3, 4, 7, 8, 64, 4096 + 2, 1 << 16};

  std::vector<unsigned char> idb(tca_rccl_unique_id_bytes());
  if (tca_rccl_get_unique_id(idb.data()) != 0) return fail("unique id", -1);
  if (tca_rccl_get_unique_id(nullptr) == 0) return fail("null id out accepted", -1);
  void* bad = reinterpret_cast<void*>(1);
  if (tca_rccl_comm_init(&bad, 2, idb.data(), 2) == 0 || bad != reinterpret_cast<void*>(1))
    return fail("rank >= nranks accepted (or comm_out written)", -1);
  if (tca_rccl_comm_init(nullptr, 2, idb.data(), 0) == 0) return fail("null comm_out accepted", -1);
  if (tca_rccl_async_error(nullptr) == 0) return fail("null comm async error", -1);
  if (tca_rccl_group_p2p(nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr) == 0)
    return fail("null comm accepted", -1);

  for (int it = 0; it < iters; ++it) {
    const int nranks = pick(1, 8);
    void* comm = nullptr;
    if (tca_rccl_comm_init(&comm, nranks, idb.data(), pick(0, nranks - 1)) != 0) return fail("init", it);
    int cnt = 0;
    if (tca_rccl_comm_count(comm, &cnt) != 0 || cnt != nranks) return fail("count", it);
    if (tca_rccl_async_error(comm) != 0) return fail("async error", it);

    const int n = pick(0, 12);
    std::vector<int> kind(n), peer(n);
    std::vector<int64_t> bytes(n);
    std::vector<void*> buf(n), alloc(n);
    bool valid = true;
    for (int i = 0; i < n; ++i) {
      kind[i] = pick(0, 40) == 0 ? (pick(0, 1) ? 2 : -1) : pick(0, 1);
      peer[i] = pick(0, 30) == 0 ? (pick(0, 1) ? -1 : nranks) : pick(0, nranks - 1);
      bytes[i] = sizes[pick(0, 9)];
      const bool null_buf = pick(0, 50) == 0;
      const bool misalign = pick(0, 3) == 0;
      alloc[i] = nullptr;
      buf[i] = nullptr;
      if (!null_buf && bytes[i] > 0) {
        // exactly bytes[i] usable bytes at buf[i]: any over-count is a heap overflow
        alloc[i] = std::malloc((size_t)bytes[i] + (misalign ? 1 : 0));
        buf[i] = static_cast<unsigned char*>(alloc[i]) + (misalign ? 1 : 0);
      }
      if (kind[i] != 0 && kind[i] != 1) valid = false;
      if (bytes[i] > 0 && (peer[i] < 0 || peer[i] >= nranks || buf[i] == nullptr)) valid = false;
    }
    g_ops.clear();
    const int groups0 = g_groups;
    const int r = tca_rccl_group_p2p(comm, n, kind.data(), peer.data(), buf.data(), bytes.data(), nullptr);
    if (g_depth != 0) return fail("group left open", it);
    if (valid) {
      if (r != 0) return fail("valid plan rejected", it);
      if (g_groups != groups0 + 1) return fail("not one group", it);
      size_t k = 0;
      for (int i = 0; i < n; ++i) {
        if (bytes[i] <= 0) continue;
        if (k >= g_ops.size()) return fail("op missing", it);
        const Op& o = g_ops[k++];
        const bool words = bytes[i] % 4 == 0 && (reinterpret_cast<uintptr_t>(buf[i]) % 4 == 0);
        if (o.kind != kind[i] || o.peer != peer[i] || o.buf != buf[i]) return fail("op order / peer", it);
        if (o.count * esize(o.dt) != (size_t)bytes[i]) return fail("byte count", it);
        if (words != (o.dt == ncclInt32)) return fail("word / byte choice", it);
      }
      if (k != g_ops.size()) return fail("extra ops", it);
    } else {
      if (r == 0) return fail("invalid plan accepted", it);
      if (!g_ops.empty() || g_groups != groups0) return fail("invalid plan posted ops", it);
    }
    // all-reduce / broadcast argument checks
    const int64_t nd = pick(0, 64);
    std::vector<double> d(nd > 0 ? nd : 1);
    if (tca_rccl_allreduce_max_f64(comm, nd > 0 ? d.data() : nullptr, nd, nullptr) != 0) return fail("allreduce", it);
    if (tca_rccl_allreduce_max_f64(comm, nullptr, 3, nullptr) == 0) return fail("allreduce null buf", it);
    const int root = pick(-1, nranks);
    const int rb = tca_rccl_broadcast(comm, d.data(), nd * 8, root, nullptr);
    if ((rb == 0) != (root >= 0 && root < nranks)) return fail("broadcast root check", it);
    for (void* p : alloc) std::free(p);
    if (tca_rccl_comm_destroy(comm) != 0) return fail("destroy", it);
  }
  std::printf("rccl plan fuzz ok: %d plans (sink %u)\n", iters, (unsigned)g_sink);
  return 0;
}
