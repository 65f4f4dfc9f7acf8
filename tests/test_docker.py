"""Container definition checks without a Docker daemon (reference
docker/server_3d/Dockerfile:43-54 builds and verifies its ops inside the image).

The Dockerfile is parsed instruction by instruction and every instruction is
checked against the tree: COPY sources exist in the build context after
.dockerignore filtering, the RUN build step's entry point exists, CMD and the
compose services' commands parse with the real CLI parsers and name models the
server can load.  A dry build stages the filtered context in a temp dir and
checks the HIP/C++ sources the image's build step would compile are all there
and that no host-built binary travels into the image."""
import fnmatch
import json
import os
import shlex
import shutil

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCKERFILE = os.path.join(ROOT, "docker", "Dockerfile")
COMPOSE = os.path.join(ROOT, "docker", "docker-compose.yml")
KEYWORDS = {"FROM", "ARG", "ENV", "WORKDIR", "COPY", "ADD", "RUN", "EXPOSE", "CMD", "ENTRYPOINT", "LABEL",
            "USER", "VOLUME", "HEALTHCHECK", "SHELL", "STOPSIGNAL", "ONBUILD"}


def parse_dockerfile(path):
    """[(KEYWORD, argument string)] with comments dropped and '\\' continuations joined."""
    out, cur = [], ""
    with open(path) as f:
        for raw in f:
            line = raw.rstrip("\n")
            if not cur and (not line.strip() or line.lstrip().startswith("#")):
                continue
            if line.endswith("\\"):
                cur += line[:-1] + " "
                continue
            cur += line
            kw, _, rest = cur.strip().partition(" ")
            out.append((kw.upper(), rest.strip()))
            cur = ""
    assert not cur, "dangling line continuation"
    return out


def dockerignore_patterns():
    with open(os.path.join(ROOT, ".dockerignore")) as f:
        return [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]


def ignored(rel, patterns):
    """Docker's matcher for the pattern forms used here: path globs, 'dir/' and '**/'."""
    parts = rel.split("/")
    for p in patterns:
        p = p.rstrip("/")
        if p.startswith("**/"):
            if any(fnmatch.fnmatch(x, p[3:]) for x in parts):
                return True
        elif "/" not in p:
            if fnmatch.fnmatch(parts[0], p) or fnmatch.fnmatch(parts[-1], p):
                return True
        elif rel == p or rel.startswith(p + "/") or fnmatch.fnmatch(rel, p):
            return True
    return False


def build_context(patterns):
    files = []
    for d, dirs, fs in os.walk(ROOT):
        rd = os.path.relpath(d, ROOT)
        dirs[:] = [x for x in dirs if not ignored(os.path.normpath(os.path.join(rd, x)).lstrip("./"), patterns)]
        for f in fs:
            rel = os.path.normpath(os.path.join(rd, f))
            if not ignored(rel, patterns):
                files.append(rel)
    return files


def test_dockerfile_instructions():
    ins = parse_dockerfile(DOCKERFILE)
    kws = [k for k, _ in ins]
    assert set(kws) <= KEYWORDS, set(kws) - KEYWORDS
    assert kws[0] in ("ARG", "FROM") and "FROM" in kws
    env = " ".join(a for k, a in ins if k == "ENV")
    for need in ("PYTORCH_ROCM_ARCH=gfx950", "TCA_OFFLOAD_ARCH=gfx950", "HSA_ENABLE_IPC_MODE_LEGACY=0"):
        assert need in env
    for k, a in ins:
        if k == "COPY":
            *srcs, _dst = shlex.split(a)
            for s in srcs:
                assert os.path.exists(os.path.join(ROOT, s)), s
    runs = [a for k, a in ins if k == "RUN"]
    assert any("requirements.txt" in r for r in runs)
    assert any("g.build()" in r and "__graft_entry__" in r for r in runs)
    text = open(DOCKERFILE).read().lower()
    assert "nvidia" not in text and "cuda" not in text  # ROCm image only


def test_dockerfile_cmd_parses():
    from triton_client_amd.server import __main__ as srv
    from triton_client_amd.server.repository import FACTORIES

    ins = dict(parse_dockerfile(DOCKERFILE))
    cmd = json.loads(ins["CMD"])
    assert cmd[:3] == ["python", "-m", "triton_client_amd.server"]
    args = srv.build_parser().parse_args(cmd[3:])
    for m in args.models.split(","):
        assert m in FACTORIES, m
    exposed = {int(p) for p in ins["EXPOSE"].split()}
    assert {args.port, args.metrics_port} <= exposed


def test_compose_services():
    from triton_client_amd.cli import main as main2d
    from triton_client_amd.cli import main3d
    from triton_client_amd.server import __main__ as srv
    from triton_client_amd.server.repository import FACTORIES

    doc = yaml.safe_load(open(COMPOSE))  # SafeLoader resolves the '<<' merge key
    svcs = doc["services"]
    assert set(svcs) == {"server", "client2d", "client3d"}
    for name, s in svcs.items():
        assert s["devices"] == ["/dev/kfd", "/dev/dri"], name  # ROCm device nodes
        assert s["environment"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        ctx = os.path.normpath(os.path.join(os.path.dirname(COMPOSE), s["build"]["context"]))
        assert ctx == ROOT and os.path.isfile(os.path.join(ctx, s["build"]["dockerfile"]))
        cmd = s["command"]
        assert cmd[0] == "python"
        if name == "server":
            assert cmd[1:3] == ["-m", "triton_client_amd.server"]
            a = srv.build_parser().parse_args(cmd[3:])
            assert a.model_repository == "/models"
            assert any(v.endswith(":/models:ro") for v in s["volumes"])
        else:
            assert os.path.isfile(os.path.join(ROOT, cmd[1])), cmd[1]
            parser = main2d if name == "client2d" else main3d
            f = parser.parse_args(cmd[2:])
            assert f.model_name in FACTORIES, f.model_name
        if name != "server":
            assert s["depends_on"] == ["server"]


def test_dry_build_context(tmp_path):
    """Stage the build context as `COPY . .` would and check the image's build
    step has every source and no host-built binary."""
    pats = dockerignore_patterns()
    for need in (".git", "build/", "triton_client_amd/_lib/", "gpurun_out/"):
        assert need in pats, need
    files = build_context(pats)
    assert not any(f.endswith((".so", ".o")) for f in files)
    assert not any(f.startswith(("build/", "gpurun_out/", ".git/", "triton_client_amd/_lib/")) for f in files)
    ctx = tmp_path / "ctx"
    for f in files:
        if f.startswith(("csrc/", "triton_client_amd/")) or f in ("__graft_entry__.py", "requirements.txt"):
            dst = ctx / f
            dst.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy2(os.path.join(ROOT, f), dst)
    for sub in ("kernels", "runtime", "include"):
        want = sorted(os.listdir(os.path.join(ROOT, "csrc", sub)))
        assert sorted(os.listdir(ctx / "csrc" / sub)) == want
    assert (ctx / "__graft_entry__.py").is_file() and (ctx / "triton_client_amd" / "_build.py").is_file()


@pytest.mark.parametrize("rel,expect", [("build/x.o", True), ("triton_client_amd/_lib/libtca_kernels.so", True),
                                        ("a/b/__pycache__/c.pyc", True), ("csrc/kernels/nms.hip", False),
                                        ("requirements.txt", False)])
def test_dockerignore_matcher(rel, expect):
    assert ignored(rel, dockerignore_patterns()) is expect
