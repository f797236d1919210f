"""Build the gfx950 library (libphdslam.so) in-tree with hipcc, and the CPU oracle.

    python cuda-phdslam_amd/build.py            # product library + driver + oracle
    python cuda-phdslam_amd/build.py --no-oracle

No cmake/ninja: each translation unit is compiled by its own hipcc call (in
parallel) to an object under build/, keyed by a SHA-256 of the compiler
command, the unit's source and every header of the tree; the objects are then
linked by one hipcc call.  An object is reused only when that key matches, so
a build always reflects the sources it is run on (no timestamps involved).
-ffp-contract=off keeps a*b+c unfused so the device rounds the way the
reference's separate multiply/add does.
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(REPO, "build", "obj")
OUT = os.path.join(HERE, "phdslam", "libphdslam.so")
SOURCES = ["phd_kernels.hip", "phd_terms.hip", "phd_eap.hip", "phd_mixed.hip", "phd_capi.hip", "phd_config.cpp", "phd_synth.cpp",
           "phd_io.cpp", "phdfilter_shim.cpp"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wno-unused-value", "-Wno-unused-result"]


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


_TOOLCHAIN = None


def _toolchain_id():
    """Compiler identity for the object cache key: `hipcc --version` (clang and
    HIP versions) and the resolved compiler path, so a toolchain upgrade at the
    same hipcc path never reuses objects built by the old one."""
    global _TOOLCHAIN
    if _TOOLCHAIN is None:
        r = subprocess.run([hipcc(), "--version"], capture_output=True, text=True)
        _TOOLCHAIN = os.path.realpath(hipcc()) + "\0" + r.stdout + r.stderr
    return _TOOLCHAIN


def _headers_digest():
    h = hashlib.sha256()
    for d in (os.path.join(REPO, "include"), CSRC):
        for f in sorted(os.listdir(d)):
            if f.endswith(".h"):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def _compile(src, defines, verbose):
    cmd = [hipcc(), f"--offload-arch={ARCH}", *FLAGS, *defines, "-I" + os.path.join(REPO, "include"), "-I" + CSRC,
           "-c", os.path.join(CSRC, src)]
    h = hashlib.sha256(" ".join(cmd).encode() + _headers_digest().encode() + _toolchain_id().encode())
    with open(os.path.join(CSRC, src), "rb") as fh:
        h.update(fh.read())
    stem = os.path.splitext(src)[0]
    obj = os.path.join(OBJ, f"{stem}-{h.hexdigest()[:16]}.o")
    if not os.path.exists(obj):
        os.makedirs(OBJ, exist_ok=True)
        _prune(stem)
        tmp = obj + f".tmp{os.getpid()}"
        if verbose:
            print(" ".join(cmd + ["-o", tmp]), flush=True)
        subprocess.run(cmd + ["-o", tmp], check=True)
        os.replace(tmp, obj)
    return obj


def _prune(stem, keep=12):
    """Bound build/obj: keep the `keep` newest objects of one source stem (the
    variants of the shipped, stamps and ablation builds live side by side)."""
    try:
        objs = [os.path.join(OBJ, f) for f in os.listdir(OBJ)
                if f.startswith(stem + "-") and f.endswith(".o") and len(f) == len(stem) + 20]
    except OSError:
        return
    objs.sort(key=lambda f: os.path.getmtime(f), reverse=True)
    for f in objs[keep:]:
        try:
            os.remove(f)
        except OSError:
            pass


def _lib_key(defines, sources=None):
    """Key of a library build: every source and header of the tree, the flags and
    the toolchain.  Written next to the library (<lib>.key) so a tree whose
    library already matches its sources (a GPU box receiving the in-tree build)
    does not compile again."""
    h = hashlib.sha256((" ".join(FLAGS + list(defines) + [ARCH])).encode() + _headers_digest().encode() +
                       _toolchain_id().encode())
    for src in sources or SOURCES:
        with open(os.path.join(CSRC, src), "rb") as fh:
            h.update(src.encode() + b"\0" + fh.read())
    return h.hexdigest()


def _up_to_date(out, key):
    try:
        with open(out + ".key") as fh:
            return os.path.exists(out) and fh.read().strip() == key
    except OSError:
        return False


def _link(out, defines, verbose):
    key = _lib_key(defines)
    if _up_to_date(out, key):
        return out
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, defines, verbose), SOURCES))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + f".tmp{os.getpid()}"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + f".tmp{os.getpid()}", out)
    with open(out + f".key.tmp{os.getpid()}", "w") as fh:
        fh.write(key + "\n")
    os.replace(out + f".key.tmp{os.getpid()}", out + ".key")
    return out


def build_lib(verbose=False):
    return _link(OUT, [], verbose)


def build_stamps_lib(verbose=False, part_a=False):
    """Diagnostic build with in-kernel phase stamps (never the shipped library):
    libphdslam_stamps.so records CPHD part C, libphdslam_stampsA.so part A."""
    out = os.path.join(HERE, "phdslam", "libphdslam_stampsA.so" if part_a else "libphdslam_stamps.so")
    return _link(out, ["-DPHD_STAMPS"] + (["-DPHD_STAMP_PART_A"] if part_a else []), verbose)


def build_ablation(xk, verbose=False):
    """Timing ablation of the workgroup update (PHD_XK in phd_kernels.hip;
    results wrong by design): libphdslam_k<xk>.so, never the shipped library."""
    out = os.path.join(HERE, "phdslam", f"libphdslam_k{xk}.so")
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, [f"-DPHD_XK={xk}"] if s == "phd_kernels.hip" else [], verbose),
                           SOURCES))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + f".tmp{os.getpid()}"]
    subprocess.run(cmd, check=True)
    os.replace(out + f".tmp{os.getpid()}", out)
    return out


def build_variant(tag, defines, verbose=False):
    """A/B variant of the workgroup update (extra -D flags on every source: the
    host's LDS layout must match the kernels'): libphdslam_v<tag>.so, never the
    shipped library."""
    out = os.path.join(HERE, "phdslam", f"libphdslam_v{tag}.so")
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, list(defines), verbose), SOURCES))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + f".tmp{os.getpid()}"]
    subprocess.run(cmd, check=True)
    os.replace(out + f".tmp{os.getpid()}", out)
    return out


def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    return os.path.join(REPO, "oracle", "liboracle.so")


def _build_exe(src, out, extra, verbose):
    """One host program (hipcc) against the in-tree libraries, skipped when its
    key (source, every header, command) matches the one stored beside it."""
    if not os.path.exists(src):
        return None
    tmp = out + f".tmp{os.getpid()}"
    cmd = [hipcc(), "-O2", "-std=c++17", "-I" + os.path.join(REPO, "include"), src, "-o", tmp,
           "-L" + os.path.dirname(OUT), *extra]
    h = hashlib.sha256((src + "|" + out + "|" + " ".join(extra)).encode() + _headers_digest().encode() +
                       _toolchain_id().encode())
    with open(src, "rb") as fh:
        h.update(fh.read())
    key = h.hexdigest()
    if _up_to_date(out, key):
        return out
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    with open(out + ".key", "w") as fh:
        fh.write(key + "\n")
    return out


GROUP_OUT = os.path.join(HERE, "phdslam", "libphdslam_group.so")


def build_group_lib(verbose=False):
    """libphdslam_group.so (include/phd_group.h): one process driving N GPUs over
    RCCL.  Its own library, so libphdslam.so (which PyTorch processes load) never
    links a second RCCL."""
    src = os.path.join(CSRC, "phd_group.cpp")
    if not os.path.exists(src):
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(rocm, "include"), src,
           "-o", GROUP_OUT + f".tmp{os.getpid()}", "-L" + os.path.dirname(OUT), "-lphdslam",
           "-L" + os.path.join(rocm, "lib"), "-lrccl", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + os.path.join(rocm, "lib")]
    h = hashlib.sha256(" ".join(c for c in cmd if ".tmp" not in c).encode() + _headers_digest().encode() +
                       _toolchain_id().encode())
    with open(src, "rb") as fh:
        h.update(fh.read())
    key = h.hexdigest()
    if _up_to_date(GROUP_OUT, key):
        return GROUP_OUT
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(GROUP_OUT + f".tmp{os.getpid()}", GROUP_OUT)
    with open(GROUP_OUT + ".key", "w") as fh:
        fh.write(key + "\n")
    return GROUP_OUT


def build_driver(verbose=False):
    """C++ drop-in driver (run_synth equivalent, and the multi-GPU sharded run
    over libphdslam_group.so) linked against libphdslam.so."""
    build_group_lib(verbose)
    return _build_exe(os.path.join(CSRC, "phdslam_run.cpp"), os.path.join(HERE, "phdslam", "phdslam_run"),
                      ["-lphdslam", "-lphdslam_group", "-Wl,-rpath,$ORIGIN"], verbose)


def build_shim_harness(verbose=False):
    """Test driver of the C++ drop-in surface (tests/shim_harness.cpp), linked
    against libphdslam.so; used only by the GPU parity tests."""
    return _build_exe(os.path.join(REPO, "tests", "shim_harness.cpp"), os.path.join(REPO, "tests", "shim_harness"),
                      ["-lphdslam", "-Wl,-rpath,$ORIGIN/../cuda-phdslam_amd/phdslam"], verbose)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="also build the PHD_STAMPS diagnostic library")
    ap.add_argument("--ablation", type=int, nargs="*", default=[], help="workgroup-update timing ablations (PHD_XK)")
    ap.add_argument("--variant", nargs="*", default=[],
                    help="A/B variants TAG:-DNAME=V[,-DNAME=V] (libphdslam_v<TAG>.so, diagnostic)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build_lib(a.verbose))
    print(build_driver(a.verbose))
    print(build_shim_harness(a.verbose))
    if a.stamps:
        print(build_stamps_lib(a.verbose))
        print(build_stamps_lib(a.verbose, part_a=True))
    for x in a.ablation:
        print(build_ablation(x, a.verbose))
    for v in a.variant:
        tag, _, defs = v.partition(":")
        print(build_variant(tag, [d for d in defs.split(",") if d], a.verbose))
    if not a.no_oracle:
        print(build_oracle())
    return 0


if __name__ == "__main__":
    sys.exit(main())
