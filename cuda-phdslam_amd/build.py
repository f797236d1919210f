"""Build the gfx950 library (libphdslam.so) in-tree with hipcc, and the CPU oracle.

    python cuda-phdslam_amd/build.py            # product library + oracle
    python cuda-phdslam_amd/build.py --no-oracle

No cmake/ninja: the product is three HIP/C++ translation units linked by one
hipcc call.  -ffp-contract=off keeps a*b+c unfused so the device rounds the
way the reference's separate multiply/add does.
"""
import argparse
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "phdslam", "libphdslam.so")
SOURCES = ["phd_kernels.hip", "phd_eap.hip", "phd_capi.hip", "phd_config.cpp", "phd_synth.cpp", "phd_io.cpp", "phdfilter_shim.cpp"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_lib(verbose=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps += [os.path.join(REPO, "include", f) for f in os.listdir(os.path.join(REPO, "include"))]
    if os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
           "-Wno-unused-value", "-Wno-unused-result", "-I" + os.path.join(REPO, "include"), "-I" + CSRC,
           *srcs, "-o", OUT]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return OUT


def build_stamps_lib(verbose=False, experiment=0):
    """Diagnostic build with in-kernel phase stamps (never the shipped library).
    experiment > 0 selects a timing ablation (results are wrong by design)."""
    out = os.path.join(HERE, "phdslam", "libphdslam_stamps.so" if not experiment else f"libphdslam_x{experiment}.so")
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
           "-DPHD_STAMPS", *([f"-DPHD_EXPERIMENT={experiment}"] if experiment else []), "-Wno-unused-value", "-Wno-unused-result", "-I" + os.path.join(REPO, "include"),
           "-I" + CSRC, *srcs, "-o", out]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    return os.path.join(REPO, "oracle", "liboracle.so")


def build_driver(verbose=False):
    """C++ drop-in driver (run_synth equivalent) linked against libphdslam.so."""
    src = os.path.join(CSRC, "phdslam_run.cpp")
    if not os.path.exists(src):
        return None
    out = os.path.join(HERE, "phdslam", "phdslam_run")
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(src), os.path.getmtime(OUT)):
        return out
    cmd = [hipcc(), "-O2", "-std=c++17", "-I" + os.path.join(REPO, "include"), src, "-o", out,
           "-L" + os.path.dirname(OUT), "-lphdslam", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="also build the PHD_STAMPS diagnostic library")
    ap.add_argument("--experiment", type=int, default=0, help="also build ablation library N (diagnostic)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build_lib(a.verbose))
    print(build_driver(a.verbose))
    if a.stamps:
        print(build_stamps_lib(a.verbose))
    if a.experiment:
        print(build_stamps_lib(a.verbose, a.experiment))
    if not a.no_oracle:
        print(build_oracle())
    return 0


if __name__ == "__main__":
    sys.exit(main())
