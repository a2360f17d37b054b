"""Build the in-tree gfx950 shared library (hipcc, no JIT cache).

    python -m stsphere.ops.build            # build if sources are newer
    python -m stsphere.ops.build --force

Produces ``ops/libstsp.so`` next to the sources, so it travels with the repo
snapshot to the GPU box.  Links roctx; RCCL is resolved at run time from the
``librccl.so.1`` the process already holds (PyTorch's copy) and its version is
checked against the API subset ``csrc/rccl_abi.h`` declares.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libstsp.so")
SOURCES = ["stage_kernel.hip", "march_kernel.hip", "march3_kernel.hip", "fused_step.hip", "tt_kernels.hip", "tt_persist.hip", "runtime.cpp"]
HEADERS = ["stsp_kernels.h", "stage_common.h", "march_common.h", "tt_common.h", "runtime.h", "rccl_abi.h"]
ARCH = os.environ.get("STSP_OFFLOAD_ARCH", "gfx950")
# library variants: "" = production; "diag" = in-kernel phase stamps of the
# stage kernel (-DSTSP_STAMPS); "xgc" = the arrival-counter hand-off of the
# xGMI halo instead of tagged granules (STSP_XG_TAG=0); the others are A/B
# switches of kept alternatives (unfused faces, block-wide panel-edge fix-up,
# own-cell wave placement, nine waves, library sqrt, compare+select slopes,
# march waves per SIMD) and the timing-only fused-step probe fp_alledge;
# xgfence: system-scope fences around the fused step's xGMI ring (multi-rank
# visibility diagnostic); xgaos: the record-major ring layout of round 5
# (STSP_XG_SOA=0), the A/B of profiles/r6_ring
VARIANT_FLAGS = {"": [], "diag": ["-DSTSP_STAMPS"], "xgc": ["-DSTSP_XG_TAG=0"],
                 "unfused": ["-DSTSP_FUSE_FACES=0"], "pe0": ["-DSTSP_PE_WAVE=0"],
                 "ownw0": ["-DSTSP_OWN_SKIP0=0"], "w9": ["-DSTSP_W10=0"], "swsqrt": ["-DSTSP_HW_SQRT=0"],
                 "selslope": ["-DSTSP_SIGN_SLOPE=0"], "wpe6": ["-DSTSP_WPE=6"], "wpe7": ["-DSTSP_WPE=7"],
                 "fp_alledge": ["-DSTSP_FPROBE_ALLEDGE=1"],
                 "xgfence": ["-DSTSP_XG_FENCE=1"], "xgaos": ["-DSTSP_XG_SOA=0"]}


def lib_for(variant: str = "") -> str:
    return LIB if not variant else os.path.join(HERE, f"libstsp_{variant}.so")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def needs_build(variant: str = "") -> bool:
    lib = lib_for(variant)
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    for f in SOURCES + HEADERS:
        p = os.path.join(CSRC, f)
        if os.path.exists(p) and os.path.getmtime(p) > t:
            return True
    return False


def _obj_dir(variant: str) -> str:
    return os.path.join(HERE, "_obj", variant or "prod")


def build(force: bool = False, verbose: bool = False, variant: str = "") -> str:
    """Compile each source to an object (in parallel; an object is rebuilt
    only when its source or a header is newer), then link the library."""
    lib = lib_for(variant)
    if not force and not needs_build(variant):
        return lib
    odir = _obj_dir(variant)
    os.makedirs(odir, exist_ok=True)
    hdr_t = max([os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS if os.path.exists(os.path.join(CSRC, h))]
                + [0.0])
    # -ffp-contract=on: a*b+c is fused only inside one source expression, so
    # every instantiation (block shape, launch-per-stage vs persistent) rounds
    # alike and multi-rank / persistent runs stay bitwise equal to one rank
    # (hipcc's default "fast" lets the backend fuse across statements, which
    # depends on the surrounding code: 8x8 blocks differed by ~1 ulp).
    flags = [f"--offload-arch={ARCH}", "-O3", "-ffp-contract=on", "-std=c++17", "-fPIC", "-Wno-unused-result",
             "-I", CSRC,
             "-I", "/opt/rocm/include", *VARIANT_FLAGS[variant]]
    objs, procs = [], []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        if not os.path.exists(sp):
            continue
        op = os.path.join(odir, src + ".o")
        objs.append(op)
        if not force and os.path.exists(op) and os.path.getmtime(op) >= max(os.path.getmtime(sp), hdr_t):
            continue
        cmd = [_hipcc(), *flags, "-c", sp, "-o", op + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        procs.append((op, cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = False
    for op, cmd, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            sys.stderr.write(out)
            failed = True
        else:
            os.replace(op + ".tmp", op)
    if failed:
        raise RuntimeError("hipcc failed")
    # RCCL is not linked: the runtime resolves it from the librccl.so.1 the
    # process already holds (PyTorch's) and checks its version (rccl_abi.h)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib + ".tmp", "-L/opt/rocm/lib",
           "-ldl", "-lrocprofiler-sdk-roctx"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"link failed ({r.returncode})")
    os.replace(lib + ".tmp", lib)
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default="", choices=sorted(VARIANT_FLAGS))
    ap.add_argument("--all", action="store_true", help="build every variant")
    a = ap.parse_args()
    for v in (sorted(VARIANT_FLAGS) if a.all else [a.variant]):
        print(build(a.force, a.verbose, v))


if __name__ == "__main__":
    main()
