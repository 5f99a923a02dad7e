"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/libblscpu.so (oracle/blscpu.c), the C restatement of the
verification path used as the large-size oracle of the GPU parity tests and as bench.py's cpu_baseline.

Only tests/, __graft_entry__ and bench.py's cpu_baseline leg import this module.  The product (lodestar_amd)
never does.  Pinned against oracle/bls12_381.py and the reference KATs by tests/test_cpu_oracle.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libblscpu.so")


class Batch(ctypes.Structure):  # include/blsgpu.h blsgpu_batch
    _fields_ = [
        ("n_sets", ctypes.c_uint32),
        ("n_jobs", ctypes.c_uint32),
        ("job_first_set", ctypes.c_void_p),
        ("job_flags", ctypes.c_void_p),
        ("pk_bytes", ctypes.c_void_p),
        ("set_pk_first", ctypes.c_void_p),
        ("pk_index", ctypes.c_void_p),
        ("msgs", ctypes.c_void_p),
        ("sigs", ctypes.c_void_p),
        ("sig_len", ctypes.c_void_p),
        ("sig_stride", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
    ]


class Stats(ctypes.Structure):
    _fields_ = [("work_requests", ctypes.c_uint32), ("batch_retries", ctypes.c_uint32),
                ("batch_sigs_success", ctypes.c_uint32), ("threads", ctypes.c_uint32)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "libblscpu.so"])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.blscpu_table_create.argtypes = [vp, u32, vp]
    lib.blscpu_table_create.restype = vp
    lib.blscpu_table_free.argtypes = [vp]
    for name in ("blscpu_sk_to_pk", "blscpu_hash_to_g2"):
        getattr(lib, name).argtypes = [u32, vp, vp, i32]
    lib.blscpu_sign.argtypes = [u32, vp, vp, vp, i32]
    lib.blscpu_sig_status.argtypes = [vp, u32]
    lib.blscpu_key_validate.argtypes = [vp, u32]
    lib.blscpu_pk_decode.argtypes = [vp, u32, vp]
    lib.blscpu_aggregate_pubkeys.argtypes = [ctypes.POINTER(Batch), vp, vp, u32, vp, i32]
    lib.blscpu_verify_jobs.argtypes = [ctypes.POINTER(Batch), vp, vp, i32, ctypes.POINTER(Stats)]
    lib.blscpu_count_get.restype = ctypes.c_uint64
    lib.blscpu_chunkify.argtypes = [u32, u32, vp, vp]
    _lib = lib
    return lib


def _buf(b):
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def sk_to_pk(sks: bytes, threads=0) -> bytes:
    """32-byte big-endian secret keys -> 96-byte uncompressed pubkeys."""
    n = len(sks) // 32
    out = np.zeros(96 * n, np.uint8)
    src = _buf(sks)
    load().blscpu_sk_to_pk(n, src.ctypes.data, out.ctypes.data, threads)
    return out.tobytes()


def sign(sks: bytes, msgs: bytes, threads=0) -> bytes:
    """(sk_i, msg_i) -> 96-byte compressed signatures sk_i H(msg_i)."""
    n = len(msgs) // 32
    out = np.zeros(96 * n, np.uint8)
    a, m = _buf(sks), _buf(msgs)
    load().blscpu_sign(n, a.ctypes.data, m.ctypes.data, out.ctypes.data, threads)
    return out.tobytes()


def hash_to_g2(msgs: bytes, threads=0) -> bytes:
    n = len(msgs) // 32
    out = np.zeros(192 * n, np.uint8)
    m = _buf(msgs)
    load().blscpu_hash_to_g2(n, m.ctypes.data, out.ctypes.data, threads)
    return out.tobytes()


def sig_status(sig: bytes) -> int:
    b = _buf(sig) if len(sig) else np.zeros(1, np.uint8)
    return load().blscpu_sig_status(b.ctypes.data, len(sig))


def key_validate(pk: bytes) -> int:
    b = _buf(pk) if len(pk) else np.zeros(1, np.uint8)
    return load().blscpu_key_validate(b.ctypes.data, len(pk))


def pk_decode(pk: bytes):
    b = _buf(pk) if len(pk) else np.zeros(1, np.uint8)
    out = np.zeros(96, np.uint8)
    st = load().blscpu_pk_decode(b.ctypes.data, len(pk), out.ctypes.data)
    return st, out.tobytes()


class Table:
    """Decoded trusted pubkey table (96-byte uncompressed entries)."""

    def __init__(self, pk96: bytes):
        lib = load()
        src = _buf(pk96)
        bad = ctypes.c_uint32(0)
        self.n = len(pk96) // 96
        self.h = lib.blscpu_table_create(src.ctypes.data, self.n, ctypes.byref(bad))
        if not self.h:
            raise ValueError(f"malformed table entry {bad.value}")

    def close(self):
        if self.h:
            load().blscpu_table_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_batch(job_first_set, sigs, sig_len, msgs, pk_bytes=None, set_pk_first=None, pk_index=None,
               job_flags=None, sig_stride=None, seed=0x4C4F444553544152):
    """blsgpu_batch from numpy/bytes arrays (same arguments as lodestar_amd.native.Context.verify_raw).
    Returns (Batch, keepalive list)."""
    jfs = np.ascontiguousarray(job_first_set, dtype=np.uint32)
    sl = np.ascontiguousarray(sig_len, dtype=np.uint32)
    n_sets = len(sl)
    sigs_a, msgs_a = _buf(sigs), _buf(msgs)
    if sig_stride is None:
        sig_stride = (len(sigs_a) // n_sets) if n_sets else 96
    keep = [jfs, sl, sigs_a, msgs_a]
    b = Batch()
    b.n_sets, b.n_jobs = n_sets, len(jfs) - 1
    b.job_first_set = jfs.ctypes.data
    if job_flags is not None:
        jf = np.ascontiguousarray(job_flags, dtype=np.uint8)
        keep.append(jf)
        b.job_flags = jf.ctypes.data
    if pk_bytes is not None:
        pk = _buf(pk_bytes)
        keep.append(pk)
        b.pk_bytes = pk.ctypes.data
    if set_pk_first is not None:
        spf = np.ascontiguousarray(set_pk_first, dtype=np.uint32)
        keep.append(spf)
        b.set_pk_first = spf.ctypes.data
    if pk_index is not None:
        pki = np.ascontiguousarray(pk_index, dtype=np.uint32)
        keep.append(pki)
        b.pk_index = pki.ctypes.data if len(pki) else 0
    b.msgs, b.sigs, b.sig_len = msgs_a.ctypes.data, sigs_a.ctypes.data, sl.ctypes.data
    b.sig_stride = sig_stride
    b.seed = seed
    return b, keep


def verify_jobs(table=None, threads=0, **batch):
    """The reference pool over one batch: (job_result int8 array, Stats)."""
    b, keep = make_batch(**batch)
    res = np.zeros(max(b.n_jobs, 1), np.int8)
    st = Stats()
    rc = load().blscpu_verify_jobs(ctypes.byref(b), table.h if table else None, res.ctypes.data, threads,
                                   ctypes.byref(st))
    if rc:
        raise RuntimeError(f"blscpu_verify_jobs -> {rc}")
    return res[: b.n_jobs], st


def aggregate_pubkeys(table=None, out_len=96, threads=0, **batch):
    """PublicKey.aggregate(set pubkeys).toBytes() per set: (bytes list, status array)."""
    b, keep = make_batch(**batch)
    out = np.zeros(out_len * max(b.n_sets, 1), np.uint8)
    st = np.zeros(max(b.n_sets, 1), np.int8)
    rc = load().blscpu_aggregate_pubkeys(ctypes.byref(b), table.h if table else None, out.ctypes.data, out_len,
                                         st.ctypes.data, threads)
    if rc:
        raise RuntimeError(f"blscpu_aggregate_pubkeys -> {rc}")
    return [out[out_len * i: out_len * (i + 1)].tobytes() for i in range(b.n_sets)], st[: b.n_sets]


def chunkify(length, min_per_chunk):
    """chunkifyMaximizeChunkSize(range(length), min_per_chunk) as the oracle applies it: list of index lists."""
    out = np.zeros(length // max(min_per_chunk, 1) + 2, np.uint32)
    nc = ctypes.c_uint32(0)
    if load().blscpu_chunkify(length, min_per_chunk, out.ctypes.data, ctypes.addressof(nc)):
        raise ValueError("blscpu_chunkify")
    return [list(range(int(out[k]), int(out[k + 1]))) for k in range(nc.value)]


def count_reset():
    load().blscpu_count_reset()


def count_get() -> int:
    return load().blscpu_count_get()
