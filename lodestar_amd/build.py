"""Builds lodestar_amd/libblsgpu.so (HIP kernels + C-ABI runtime) for gfx950 with hipcc, in-tree.

    python -m lodestar_amd.build            # incremental
    python -m lodestar_amd.build --force
"""
import hashlib
import os
import subprocess
import sys
import time

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.environ.get("BLSGPU_LIB") or os.path.join(PKG, "libblsgpu.so")  # override: tuning variants
ARCH = os.environ.get("BLSGPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["k_sig.hip", "k_msm.hip", "k_hash.hip", "k_hmap.hip", "k_pk.hip", "k_miller.hip", "k_group.hip", "k_inv.hip", "k_ssz.hip", "k_debug.hip",
           "runtime.cpp"]


OBJ_DIR = os.path.join(PKG, "build")  # per-TU objects, kept so an edit rebuilds only the TUs it touches


# Per-translation-unit defines of the product build.  BLSGPU_TU_DEFINES overrides it for experiments:
# "k_miller.hip=BLS_INLINE_PRODUCTS=1+OTHER=2;k_hash.hip=..." ("" = none).
# k_sig.hip with its decode helpers inlined (BLS_INLINE_BIG: sig_decode_point, fp2_sqrt and the (p-3)/4 power in
# the kernel, no nested call frames): k_sig_decode's private segment 1,296 -> 496 B/lane at the same throughput
# (profiles/r03_sigbig_ab.txt)
TU_DEFINES = {"k_sig.hip": ["BLS_INLINE_BIG=1"]}


def tu_defines():
    env = os.environ.get("BLSGPU_TU_DEFINES")
    if env is None:
        return TU_DEFINES
    out = {}
    for part in filter(None, env.split(";")):
        tu, _, defs = part.partition("=")
        out[tu] = [d for d in defs.split("+") if d]
    return out


# Per-TU compiler flags.  The pubkey stage schedules for ILP (LLVM's max-ILP strategy): its kernels run one wave per
# SIMD, so occupancy-driven scheduling buys nothing there (round 4: hash + pubkey TUs C2 +1.5% at 20 steps, +1.7% at
# 100; the same strategy on every TU lost 6%: the Miller accumulation and the decode spill more under it).  Round 6:
# the hash TUs' kernels now run two waves per SIMD (lane pairs), where max-ILP only raises register pressure: the
# cofactor clearing (k_hash.hip) schedules for minimum registers (k_hash_clear2 713 -> 366 spilled VGPRs, 848 -> 496 B
# of scratch per lane) and the maps (k_hmap.hip) with the default scheduler (k_hash_map 214 -> 98, 1,984 -> 1,664 B);
# C2 equal within noise (3.40M vs 3.39M at 20 steps, 3.83M vs 3.84M at 100; profiles/r06_hash_sched_ab.json).
_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
_MINREG = ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]
TU_CFLAGS = {"k_hash.hip": _MINREG, "k_pk.hip": _ILP}


def tu_cflags():
    """Per-TU extra compiler flags; BLSGPU_TU_CFLAGS="k_hash.hip=-mllvm -flag;k_x.hip=..." overrides (tuning)."""
    env = os.environ.get("BLSGPU_TU_CFLAGS")
    if env is None:
        return TU_CFLAGS
    out = {}
    for part in filter(None, env.split(";")):
        tu, _, flags = part.partition("=")
        out[tu] = flags.split()
    return out


def _headers():
    out = [os.path.join(ROOT, "include", "blsgpu.h")]
    for f in os.listdir(CSRC):
        if f.endswith((".hpp", ".h")):
            out.append(os.path.join(CSRC, f))
    return out


def _tu_deps(src):
    """runtime.cpp sees only the C-ABI header and the kernel launch declarations; a kernel TU sees every
    arithmetic header."""
    if src.endswith(".cpp"):
        return [os.path.join(CSRC, src), os.path.join(CSRC, "kernels.h"), os.path.join(CSRC, "batch_rand.hpp"),
                os.path.join(ROOT, "include", "blsgpu.h")]
    return [os.path.join(CSRC, src)] + _headers()


def _deps():
    # (this file too: its per-TU defines change the objects)
    return _headers() + [os.path.join(CSRC, s) for s in SOURCES] + [os.path.abspath(__file__)]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force=False, verbose=True):
    if not force and up_to_date():
        build_node_addon(verbose=verbose)
        return LIB
    objs = []
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include")]
    defines = os.environ.get("BLSGPU_DEFINES", "").split()  # e.g. BLSGPU_WPE=2
    common += ["-D" + d for d in defines]
    cflags = os.environ.get("BLSGPU_CFLAGS", "").split()  # tuning variants: extra compiler flags
    common += cflags
    tu_defs = tu_defines()
    os.makedirs(OBJ_DIR, exist_ok=True)
    # objects are keyed by the library name and the defines, so variant builds never reuse each other's objects
    key = os.path.splitext(os.path.basename(LIB))[0] + ("." + "_".join(defines).replace("=", "-") if defines else "")
    if cflags:
        key += ".cf" + hashlib.md5(" ".join(cflags).encode()).hexdigest()[:8]
    # one translation unit per pipeline stage, compiled in parallel (the stage kernels are large)
    procs = []
    t0 = time.time()
    for src in SOURCES:
        tdefs = tu_defs.get(src, [])
        tflags = tu_cflags().get(src, [])
        obj = os.path.join(OBJ_DIR, key + "." + os.path.splitext(src)[0] +
                           ("." + "_".join(tdefs).replace("=", "-") if tdefs else "") +
                           (".cf" + hashlib.md5(" ".join(tflags).encode()).hexdigest()[:8] if tflags else "") + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in _tu_deps(src)):
            continue
        cmd = [HIPCC] + common + ["-D" + d for d in tdefs] + tflags + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd)))
    for src, p in procs:
        if p.wait() != 0:
            raise RuntimeError(f"hipcc failed on {src}")
        if verbose:
            print(f"  {src}: done at {time.time() - t0:.0f} s", flush=True)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", LIB] + objs + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    build_node_addon(verbose=verbose)
    return LIB


NODE_DIR = os.path.join(PKG, "node")
ADDON = os.path.join(NODE_DIR, "blsgpu_napi.node")
NODE_INC = "/usr/include/node"


def build_node_addon(force=False, verbose=True):
    """The N-API addon (lodestar_amd/node/blsgpu_napi.c) the JS BlsGpuVerifier loads.  Plain gcc against the
    system node headers; links libblsgpu.so from the package directory (rpath $ORIGIN/..).  Skipped when the
    node headers are absent."""
    src = os.path.join(NODE_DIR, "blsgpu_napi.c")
    if not os.path.exists(os.path.join(NODE_INC, "node_api.h")):
        if verbose:
            print("node headers not found: N-API addon not built", flush=True)
        return None
    if not force and os.path.exists(ADDON) and os.path.getmtime(ADDON) >= max(
            os.path.getmtime(src), os.path.getmtime(LIB), os.path.getmtime(os.path.join(ROOT, "include", "blsgpu.h"))):
        return ADDON
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wno-unused-parameter", "-shared", "-fPIC",
           "-DNODE_GYP_MODULE_NAME=blsgpu_napi", "-I", NODE_INC, "-I", os.path.join(ROOT, "include"), src,
           "-o", ADDON, "-L", PKG, "-l:libblsgpu.so", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return ADDON


if __name__ == "__main__":
    build(force="--force" in sys.argv)
