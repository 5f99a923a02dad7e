"""ctypes wrapper for tests/native/libbls_emu.so (host build of the device arithmetic, test-only)."""
import ctypes
import os
import subprocess

from oracle import bls12_381 as bls

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "emu.cpp")
LIB = os.path.join(HERE, "native", "libbls_emu.so")
CSRC = os.path.join(os.path.dirname(HERE), "lodestar_amd", "csrc")


def build_emu():
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return LIB
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", LIB, SRC])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build_emu())
        _lib.emu_g2_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        _lib.emu_g1_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        _lib.emu_sig_decode.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    return _lib


def fpb(x):
    return (x % bls.P).to_bytes(48, "big")


def fromb(b):
    return int.from_bytes(b, "big")


def f2b(a):
    return fpb(a[1]) + fpb(a[0])


def b2f2(b):
    return (fromb(b[48:96]), fromb(b[0:48]))


def g1b(p):
    return fpb(p[0]) + fpb(p[1])


def g2b(p):
    return f2b(p[0]) + f2b(p[1])


def b2g2(b):
    return (b2f2(b[:96]), b2f2(b[96:]))


def b2g1(b):
    return (fromb(b[:48]), fromb(b[48:]))


def f12b(f):
    out = b""
    for c6 in f:
        for c2 in c6:
            out += fpb(c2[0]) + fpb(c2[1])
    return out


def b2f12(b):
    vals = [fromb(b[48 * i : 48 * i + 48]) for i in range(12)]
    c2 = [(vals[2 * i], vals[2 * i + 1]) for i in range(6)]
    return ((c2[0], c2[1], c2[2]), (c2[3], c2[4], c2[5]))


LAMBDA = None


def r_of_word(w, raw=False):
    """Batch scalar of a 64-bit word (runtime.cpp / k_common.hpp jac_mul_scalar_word): r = a + b lambda mod the
    group order, lambda = -z^2 (phi on G1, -psi^2 on G2), a = 2 lo + 1 - 2^32, b = 2 hi + 1 - 2^32 of the word's
    32-bit halves; word 0 = r = 1 (CoreVerify) unless `raw` (the digits' value, as jac_mul_scalar_word computes)."""
    from oracle import bls12_381 as bls

    if w == 0 and not raw:
        return 1
    z = 0xD201000000010000
    lam = (-z * z) % bls.R
    a = 2 * (w & 0xFFFFFFFF) + 1 - 2**32
    b = 2 * (w >> 32) + 1 - 2**32
    return (a + b * lam) % bls.R
