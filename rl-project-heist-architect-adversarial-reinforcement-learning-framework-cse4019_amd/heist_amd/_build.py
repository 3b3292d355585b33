"""Builds libheist_hip.so (the C ABI of include/heist.h) for gfx950, in-tree.

hipcc compiles each csrc/*.hip with -ffp-contract=off (the env kernels must not fuse
multiplies into adds: the reference's raycast relies on separately rounded IEEE
operations) and the library is linked against the HIP runtime that torch ships, so
that torch tensors' device pointers and streams are valid inside it.
"""
import hashlib
import os
import re
import subprocess
import sys

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
# HEIST_LIB: load another build of the library (A/B measurements of compile-time variants)
LIB_PATH = os.environ.get("HEIST_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libheist_hip.so")
BUILD_DIR = os.path.join(PKG_ROOT, "build")
ARCH = os.environ.get("HEIST_OFFLOAD_ARCH", "gfx950")
SOURCES = ["heist_env.hip", "heist_arch.hip", "heist_arch_update.hip", "heist_ppo.hip", "heist_policy.hip", "heist_train.hip",
           "heist_train_conv.hip", "heist_capi.hip"]
# headers are found per source by following its #include "..." lines (_includes)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# heist_env.hip: no SLP vectorization -- ROCm 7.2 clang miscompiles the packed-fp32
# (v_pk_*_f32) forms of the fast raycast (see the fast path notes in heist_env.hip).  No
# machine LICM: it hoists the raycast's literal constants (the sin/cos polynomial
# coefficients, lane masks) out of the K-tick loop of step_multi_kernel and the chunk loops,
# where they stay live in VGPRs across every other phase: 175 VGPRs spilled in
# step_multi_kernel<2,4,8,1024> with it, 46 (reloaded once per tick) without; the
# single-tick step kernel drops from 64 VGPRs + 3 spilled to 53 with none.
# HEIST_ENV_FLAGS replaces this list (A/B builds).
FILE_FLAGS = {"heist_env.hip": os.environ.get("HEIST_ENV_FLAGS", "-fno-slp-vectorize -mllvm -disable-machine-licm").split(),
              # no SLP: packed-fp32 VALU beside MFMAs costs issue slots (MI355X_MICROARCH.md);
              # solver_conv_kernel<20,20> 19.9K -> 19.2K cycles per env (r04r stamps)
              "heist_policy.hip": os.environ.get("HEIST_POLICY_FLAGS", "-fno-slp-vectorize").split(),  # A/B builds
              # the persistent Architect update: machine LICM would keep loop-invariant scalars of
              # every phase live across the whole step loop (SGPR spills 267 -> 132 without it)
              "heist_arch_update.hip": ["-mllvm", "-disable-machine-licm"]}
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
          "--offload-arch=" + ARCH, "-I", INCLUDE, "-I", CSRC]


def _torch_lib_dir():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    return d if os.path.exists(os.path.join(d, "libamdhip64.so")) else None


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


_INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _includes(path, seen=None):
    """Every quoted header path reaches through #include "..." (csrc/ and include/), so a
    generated header (heist_fan_intervals.h, heist_sincos_table.h) rebuilds its users."""
    seen = set() if seen is None else seen
    try:
        with open(path) as f:
            text = f.read()
    except OSError:
        return seen
    for name in _INCLUDE_RE.findall(text):
        for d in (os.path.dirname(path), CSRC, INCLUDE):
            p = os.path.join(d, name)
            if os.path.exists(p):
                if p not in seen:
                    seen.add(p)
                    _includes(p, seen)
                break
    return seen


def _command(src, obj):
    return [HIPCC] + CFLAGS + FILE_FLAGS.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]


def _build_dir():
    """Objects of the product library in build/, of any other library (HEIST_LIB) or flag
    set in a directory of their own, so a variant build never links or overwrites the
    product's objects."""
    if not os.environ.get("HEIST_LIB"):
        return BUILD_DIR
    return os.path.join(BUILD_DIR, "variant_" + hashlib.sha1(LIB_PATH.encode()).hexdigest()[:12])


def needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    deps = {__file__}
    for src in SOURCES:
        deps.add(os.path.join(CSRC, src))
        deps |= _includes(os.path.join(CSRC, src))
    if max(_mtime(d) for d in deps) > _mtime(LIB_PATH):
        return True
    bd = _build_dir()
    return any(_cmd_changed(src, os.path.join(bd, src.replace(".hip", ".o"))) for src in SOURCES)


def _cmd_file(obj):
    return obj + ".cmd"


def _cmd_changed(src, obj):
    """The object was compiled with another command line (flags from HEIST_*_FLAGS or
    HEIST_OFFLOAD_ARCH), recorded beside it."""
    try:
        with open(_cmd_file(obj)) as f:
            return f.read() != " ".join(_command(src, obj))
    except OSError:
        return True


def _stale(src, obj):
    """obj needs compiling: older than its source or any header it includes, or built with
    another command line.  heist_env.hip alone takes ~4 min, so an edit elsewhere does not
    rebuild it."""
    deps = [os.path.join(CSRC, src)] + sorted(_includes(os.path.join(CSRC, src)))
    return max(_mtime(d) for d in deps) > _mtime(obj) or _cmd_changed(src, obj)


def build(force=False, verbose=False, jobs=4):
    if not force and not needs_build():
        return LIB_PATH
    bd = _build_dir()
    os.makedirs(bd, exist_ok=True)
    procs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(bd, src.replace(".hip", ".o"))
        objs.append(obj)
        if not force and not _stale(src, obj):
            continue
        cmd = _command(src, obj)
        if os.path.exists(_cmd_file(obj)):
            os.remove(_cmd_file(obj))
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, obj, cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        running = [p for _, _, _, p in procs if p.poll() is None]
        if len(running) >= jobs:
            running[0].wait()
    for src, obj, cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s" % (src, out.decode(errors="replace")))
        with open(_cmd_file(obj), "w") as f:
            f.write(" ".join(cmd))
        if verbose and out:
            print(out.decode(errors="replace"), file=sys.stderr)
    tl = _torch_lib_dir()
    link = ["g++", "-shared", "-o", LIB_PATH + ".tmp"] + objs
    if tl:
        link += ["-L" + tl, "-l:libamdhip64.so", "-Wl,-rpath," + tl]
    else:
        link += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
