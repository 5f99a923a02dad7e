"""lodestar_amd: MI355X-native BLS12-381 signature-set verifier (drop-in for Lodestar's IBlsVerifier path).

The product is libblsgpu.so (HIP kernels + C-ABI runtime, include/blsgpu.h); this package holds its
sources (csrc/), the build script, the ctypes binding (native.py) and the Python mirror of the
reference's IBlsVerifier interface (verifier.py)."""
__all__ = ["native", "build"]
