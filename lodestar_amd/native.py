"""ctypes binding of libblsgpu.so (include/blsgpu.h).  Loads the in-tree library and fails loudly if it
is missing -- there is no CPU fallback for verification."""
import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLSGPU_LIB") or os.path.join(PKG, "libblsgpu.so")  # override: tuning variants

# job / status codes (blsgpu_code)
OK = 0
BAD_ENCODING = 1
POINT_NOT_ON_CURVE = 2
POINT_NOT_IN_GROUP = 3
PK_IS_INFINITY = 6
INVALID_SIZE = 8
EMPTY_AGGREGATE = 9
EMPTY_SET = 10
DEVICE_ERROR = 11
ERR_ARGS = 100
ERR_NO_DEVICE = 101
ERR_CLOSED = 102
ERR_ENTROPY = 103
# blsgpu_batch.job_flags bits
JOB_BATCHABLE = 1
JOB_URGENT = 2  # VerifySignatureOpts.verifyOnMainThread: the device's urgent lane
# blsgpu_debug_inject targets
INJECT_ENTROPY = 1
INJECT_DEVICE = 2

EXPORTED_SYMBOLS = [
    "blsgpu_init",
    "blsgpu_destroy",
    "blsgpu_device_count",
    "blsgpu_pubkeys_upload",
    "blsgpu_pubkeys_count",
    "blsgpu_verify",
    "blsgpu_submit",
    "blsgpu_set_option",
    "blsgpu_code_name",
    "blsgpu_debug_op",
    "blsgpu_aggregate_pubkeys",
    "blsgpu_key_validate",
    "blsgpu_signing_roots",
    "blsgpu_shard_jobs",
    "blsgpu_get_option",
    "blsgpu_chunkify",
    "blsgpu_batch_scalars",
    "blsgpu_debug_inject",
    "blsgpu_route_call",
]
ROOT_OBJECT = 0
ROOT_ATTESTATION_DATA = 1


class Batch(ctypes.Structure):
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
    _fields_ = [
        ("groups", ctypes.c_uint32),
        ("batch_retries", ctypes.c_uint32),
        ("batch_sigs_success", ctypes.c_uint32),
        ("devices_used", ctypes.c_uint32),
        ("device_ms", ctypes.c_double),
        ("stage_ms", ctypes.c_double * 8),
        ("unique_messages", ctypes.c_uint32),
        ("pairing_units", ctypes.c_uint32),
        ("miller_chunks", ctypes.c_uint32),
        ("run_sets", ctypes.c_uint32),
        ("run_calls", ctypes.c_uint32),
        ("fallback_jobs", ctypes.c_uint32),
        ("fallback_miller", ctypes.c_uint32),
        ("urgent_lane", ctypes.c_uint32),
        ("host_ms", ctypes.c_double),
    ]


STAGES = ["sig_decode", "hash_to_g2", "pk_aggregate", "pk_finish", "sig_msm", "miller_sets",
          "group_reduce", "group_check"]
# the kernels each stage's HIP-event interval covers (rocprof lists them separately; k_batch_inv runs in both the
# hash and the pubkey stage)
KERNEL_OF_STAGE = ["k_sig_decode+k_sig_subgroup2+k_sig_subgroup_coop",
                   "k_hash_prep+k_batch_inv+k_hash_map+k_hash_clear+k_hash_clear2+k_hash_clear_coop+k_h_affine",
                   "k_pk_aggregate+k_pk_aggregate_g", "k_pk_finish+k_batch_inv+k_pk_affine",
                   "k_job_mask+k_msm_bucket+k_msm_bucket2+k_msm_slice_pairs+k_msm_slice_pairs2+k_msm_window+k_msm_window2"
                   "+k_msm_horner+k_msm_horner_lane",
                   "k_miller_lines+k_miller_lines2+k_miller_acc+k_miller_acc2+k_miller_acc6+k_miller_accx+k_miller_coop",
                   "k_f_runs+k_f_pairs+k_f_gather", "k_group_sig_miller+k_group_check"]


DONE_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -m lodestar_amd.build` (hipcc, gfx950). "
            "There is no CPU verification path."
        )
    lib = ctypes.CDLL(LIB_PATH)
    lib.blsgpu_init.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.blsgpu_init.restype = ctypes.c_int
    lib.blsgpu_destroy.argtypes = [ctypes.c_void_p]
    lib.blsgpu_destroy.restype = None
    lib.blsgpu_device_count.argtypes = [ctypes.c_void_p]
    lib.blsgpu_device_count.restype = ctypes.c_int
    lib.blsgpu_pubkeys_upload.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
    lib.blsgpu_pubkeys_upload.restype = ctypes.c_int
    lib.blsgpu_pubkeys_count.argtypes = [ctypes.c_void_p]
    lib.blsgpu_pubkeys_count.restype = ctypes.c_uint32
    lib.blsgpu_verify.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch), ctypes.c_void_p, ctypes.POINTER(Stats)]
    lib.blsgpu_verify.restype = ctypes.c_int
    lib.blsgpu_submit.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch), ctypes.c_void_p, ctypes.POINTER(Stats),
                                  DONE_CB, ctypes.c_void_p]
    lib.blsgpu_submit.restype = ctypes.c_int
    lib.blsgpu_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
    lib.blsgpu_set_option.restype = ctypes.c_int
    lib.blsgpu_code_name.argtypes = [ctypes.c_int]
    lib.blsgpu_code_name.restype = ctypes.c_char_p
    lib.blsgpu_debug_op.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                    ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    lib.blsgpu_debug_op.restype = ctypes.c_int
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.blsgpu_aggregate_pubkeys.argtypes = [vp, ctypes.POINTER(Batch), vp, u32, vp]
    lib.blsgpu_key_validate.argtypes = [vp, u32, vp, u32, u32, vp, vp]
    lib.blsgpu_signing_roots.argtypes = [vp, ctypes.c_int, u32, vp, u32, vp, u32, vp]
    lib.blsgpu_shard_jobs.argtypes = [vp, vp, u32, u32, vp]
    lib.blsgpu_get_option.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
    lib.blsgpu_chunkify.argtypes = [u32, u32, vp, vp]
    lib.blsgpu_batch_scalars.argtypes = [ctypes.POINTER(Batch), vp]
    lib.blsgpu_batch_scalars.restype = ctypes.c_int
    lib.blsgpu_debug_inject.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
    lib.blsgpu_debug_inject.restype = ctypes.c_int
    lib.blsgpu_route_call.argtypes = [u32, u32, vp, ctypes.c_int64, u32, vp, vp]
    lib.blsgpu_route_call.restype = ctypes.c_int
    _lib = lib
    return lib


def code_name(code: int) -> str:
    n = load().blsgpu_code_name(code)
    return n.decode() if n else f"BLSGPU_{code}"


def shard_jobs(job_first_set, n_parts, set_pk_first=None):
    """The runtime's sharding rule (C-ABI blsgpu_shard_jobs, pure host code): [(job_begin, job_end)]."""
    jfs = np.ascontiguousarray(job_first_set, dtype=np.uint32)
    spf = None if set_pk_first is None else np.ascontiguousarray(set_pk_first, dtype=np.uint32)
    out = np.zeros(n_parts + 1, np.uint32)
    rc = load().blsgpu_shard_jobs(jfs.ctypes.data, None if spf is None else spf.ctypes.data, len(jfs) - 1, n_parts,
                                  out.ctypes.data)
    if rc != OK:
        raise ValueError(f"blsgpu_shard_jobs -> {code_name(rc)}")
    return [(int(out[k]), int(out[k + 1])) for k in range(n_parts)]


def route_call(n_sets, device_load, split_sets=16384, start=0):
    """The runtime's call routing (C-ABI blsgpu_route_call, pure host code): the devices, in shard order, a call of
    n_sets sets runs on given each device's queued cost."""
    dl = np.ascontiguousarray(device_load, dtype=np.int64)
    out = np.zeros(max(len(dl), 1), np.uint32)
    k = ctypes.c_uint32(0)
    rc = load().blsgpu_route_call(n_sets, len(dl), dl.ctypes.data, split_sets, start, out.ctypes.data,
                                  ctypes.addressof(k))
    if rc != OK:
        raise ValueError(f"blsgpu_route_call -> {code_name(rc)}")
    return [int(x) for x in out[: k.value]]


def chunkify(length, min_per_chunk):
    """chunkifyMaximizeChunkSize(range(length), min_per_chunk) (reference multithread/utils.ts:4-19) through the
    C-ABI (blsgpu_chunkify, pure host code): list of index lists."""
    out = np.zeros(length // max(min_per_chunk, 1) + 2, np.uint32)
    nc = ctypes.c_uint32(0)
    rc = load().blsgpu_chunkify(length, min_per_chunk, out.ctypes.data, ctypes.addressof(nc))
    if rc != OK:
        raise ValueError(f"blsgpu_chunkify -> {code_name(rc)}")
    return [list(range(int(out[k]), int(out[k + 1]))) for k in range(nc.value)]


def batch_scalars(job_first_set, job_flags=None, seed=0):
    """The batch scalar words a call would use (C-ABI blsgpu_batch_scalars, pure host code): uint64 array, one word
    per set (0 = r = 1).  Raises RuntimeError(ERR_ENTROPY) when seed is 0 and the OS gives no randomness."""
    jfs = np.ascontiguousarray(job_first_set, dtype=np.uint32)
    if len(jfs) == 0:
        raise ValueError("job_first_set needs n_jobs + 1 >= 1 entries")
    n = int(jfs[-1])
    b = Batch()
    b.n_sets = n
    b.n_jobs = len(jfs) - 1
    b.job_first_set = jfs.ctypes.data
    keep = [jfs]
    if job_flags is not None:
        fl = np.ascontiguousarray(job_flags, dtype=np.uint8)
        keep.append(fl)
        b.job_flags = fl.ctypes.data
    b.seed = seed
    out = np.zeros(max(n, 1), np.uint64)
    rc = load().blsgpu_batch_scalars(ctypes.byref(b), out.ctypes.data)
    if rc != OK:
        raise RuntimeError(f"blsgpu_batch_scalars -> {code_name(rc)}")
    return out[:n]


def debug_inject(what, skip=0, count=1):
    """Arms the library's fault injection (blsgpu_debug_inject): after `skip` more events, the next `count` entropy
    draws (INJECT_ENTROPY) or pipeline runs (INJECT_DEVICE) fail.  count 0 disarms."""
    rc = load().blsgpu_debug_inject(what, skip, count)
    if rc != OK:
        raise ValueError(f"blsgpu_debug_inject -> {code_name(rc)}")


def _u8(b):
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)


def make_batch(job_first_set, sigs, sig_len, msgs, pk_bytes=None, set_pk_first=None, pk_index=None,
               job_flags=None, sig_stride=None, seed=0x4C4F444553544152):
    """blsgpu_batch over numpy/bytes arrays: (Batch, keep-alive list).  Modes: pk_bytes alone (one key per
    set), pk_bytes + set_pk_first (bytes aggregate), set_pk_first + pk_index (device table)."""
    job_first_set = np.ascontiguousarray(job_first_set, dtype=np.uint32)
    sig_len = np.ascontiguousarray(sig_len, dtype=np.uint32)
    n_sets = len(sig_len)
    sigs, msgs = _u8(sigs), _u8(msgs)
    if sig_stride is None:
        sig_stride = (len(sigs) // n_sets) if n_sets else 96
    keep = [job_first_set, sig_len, sigs, msgs]
    b = Batch()
    b.n_sets = n_sets
    b.n_jobs = len(job_first_set) - 1
    b.job_first_set = job_first_set.ctypes.data
    if job_flags is not None:
        job_flags = np.ascontiguousarray(job_flags, dtype=np.uint8)
        keep.append(job_flags)
        b.job_flags = job_flags.ctypes.data
    if pk_bytes is not None:
        pk = _u8(pk_bytes)
        if len(pk) == 0:
            pk = np.zeros(1, np.uint8)
        keep.append(pk)
        b.pk_bytes = pk.ctypes.data
    if set_pk_first is not None:
        set_pk_first = np.ascontiguousarray(set_pk_first, dtype=np.uint32)
        keep.append(set_pk_first)
        b.set_pk_first = set_pk_first.ctypes.data
    if pk_index is not None:
        pk_index = np.ascontiguousarray(pk_index, dtype=np.uint32)
        keep.append(pk_index)
        b.pk_index = pk_index.ctypes.data if len(pk_index) else set_pk_first.ctypes.data
    b.msgs = msgs.ctypes.data if len(msgs) else 0
    b.sigs = sigs.ctypes.data if len(sigs) else 0
    b.sig_len = sig_len.ctypes.data if len(sig_len) else 0
    b.sig_stride = sig_stride
    b.seed = seed
    return b, keep


class Pending:
    """An asynchronous call of Context.submit_raw."""

    status = None
    t_done = None

    def wait(self, timeout=None):
        if not self.ev.wait(timeout):
            raise TimeoutError("blsgpu_submit: call not completed")
        if self.status != OK:
            raise RuntimeError(f"blsgpu_submit -> {code_name(self.status)}")
        return self.res[: self.n_jobs], self.st


class Context:
    """Owns a blsgpu_ctx on one or more HIP devices."""

    def __init__(self, devices=None):
        lib = load()
        self._lib = lib
        h = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = lib.blsgpu_init(arr, len(devices), ctypes.byref(h))
        else:
            rc = lib.blsgpu_init(None, 0, ctypes.byref(h))
        if rc != OK:
            raise RuntimeError(f"blsgpu_init failed: {code_name(rc)} (no usable MI355X?)")
        self.h = h

    def close(self):
        if self.h:
            self._lib.blsgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_count(self):
        return self._lib.blsgpu_device_count(self.h)

    def set_option(self, key: str, value: int):
        rc = self._lib.blsgpu_set_option(self.h, key.encode(), int(value))
        if rc != OK:
            raise ValueError(f"blsgpu_set_option({key}) -> {code_name(rc)}")

    def get_option(self, key: str) -> int:
        v = ctypes.c_int64(0)
        rc = self._lib.blsgpu_get_option(self.h, key.encode(), ctypes.byref(v))
        if rc != OK:
            raise ValueError(f"blsgpu_get_option({key}) -> {code_name(rc)}")
        return v.value

    def upload_pubkeys(self, first_index: int, pk96: bytes):
        n = len(pk96) // 96
        rc = self._lib.blsgpu_pubkeys_upload(self.h, first_index, pk96, n)
        if rc != OK:
            raise ValueError(f"blsgpu_pubkeys_upload -> {code_name(rc)}")

    @property
    def pubkeys_count(self):
        return self._lib.blsgpu_pubkeys_count(self.h)

    def verify_raw(self, job_first_set, sigs, sig_len, msgs, pk_bytes=None, set_pk_first=None, pk_index=None,
                   job_flags=None, sig_stride=None, seed=0x4C4F444553544152):
        """Low-level call: numpy/bytes arrays in, (job_result int8 array, Stats) out."""
        b, keep = make_batch(job_first_set, sigs, sig_len, msgs, pk_bytes, set_pk_first, pk_index, job_flags,
                             sig_stride, seed)
        res = np.zeros(max(b.n_jobs, 1), dtype=np.int8)
        st = Stats()
        rc = self._lib.blsgpu_verify(self.h, ctypes.byref(b), res.ctypes.data, ctypes.byref(st))
        if rc != OK:
            raise RuntimeError(f"blsgpu_verify -> {code_name(rc)}")
        return res[: b.n_jobs], st

    def submit_raw(self, job_first_set, sigs, sig_len, msgs, pk_bytes=None, set_pk_first=None, pk_index=None,
                   job_flags=None, sig_stride=None, seed=0x4C4F444553544152):
        """Asynchronous call (blsgpu_submit: inputs copied before it returns): a Pending whose wait() gives
        (job_result int8 array, Stats) once the runtime's done callback ran."""
        import threading

        b, keep = make_batch(job_first_set, sigs, sig_len, msgs, pk_bytes, set_pk_first, pk_index, job_flags,
                             sig_stride, seed)
        p = Pending()
        p.res = np.zeros(max(b.n_jobs, 1), dtype=np.int8)
        p.n_jobs = b.n_jobs
        p.st = Stats()
        p.ev = threading.Event()

        def done(user, status):
            p.status = status
            p.t_done = __import__("time").perf_counter()
            p.ev.set()

        p.cb = DONE_CB(done)  # kept alive with the Pending until the callback ran
        rc = self._lib.blsgpu_submit(self.h, ctypes.byref(b), p.res.ctypes.data, ctypes.byref(p.st), p.cb, None)
        if rc != OK:
            raise RuntimeError(f"blsgpu_submit -> {code_name(rc)}")
        return p

    def aggregate_pubkeys(self, pk_bytes=None, set_pk_first=None, pk_index=None, out_len=96):
        """PublicKey.aggregate(...).toBytes() per set on the GPU: (list of bytes, status int8 array)."""
        n = (len(set_pk_first) - 1) if set_pk_first is not None else len(pk_bytes) // 96
        b, keep = make_batch(np.array([0, n]), b"", np.zeros(n, np.uint32), b"", pk_bytes, set_pk_first, pk_index)
        out = np.zeros(max(n, 1) * out_len, np.uint8)
        st = np.zeros(max(n, 1), np.int8)
        rc = self._lib.blsgpu_aggregate_pubkeys(self.h, ctypes.byref(b), out.ctypes.data, out_len, st.ctypes.data)
        if rc != OK:
            raise RuntimeError(f"blsgpu_aggregate_pubkeys -> {code_name(rc)}")
        return [out[out_len * i: out_len * (i + 1)].tobytes() for i in range(n)], st[:n]

    def key_validate(self, pks: bytes, pk_len: int):
        """KeyValidate on the GPU: (96-byte uncompressed keys, status int8 array)."""
        n = len(pks) // pk_len
        src = _u8(pks)
        out = np.zeros(max(n, 1) * 96, np.uint8)
        st = np.zeros(max(n, 1), np.int8)
        rc = self._lib.blsgpu_key_validate(self.h, n, src.ctypes.data, pk_len, pk_len, out.ctypes.data, st.ctypes.data)
        if rc != OK:
            raise RuntimeError(f"blsgpu_key_validate -> {code_name(rc)}")
        return out[: 96 * n].tobytes(), st[:n]

    def signing_roots(self, kind: int, objects: bytes, domains: bytes):
        """computeSigningRoot on the GPU: one domain for all (32 B) or one per object."""
        obj_len = 32 if kind == ROOT_OBJECT else 128
        n = len(objects) // obj_len
        o, d = _u8(objects), _u8(domains)
        dstride = 0 if len(domains) == 32 else 32
        out = np.zeros(max(n, 1) * 32, np.uint8)
        rc = self._lib.blsgpu_signing_roots(self.h, kind, n, o.ctypes.data, obj_len, d.ctypes.data, dstride,
                                            out.ctypes.data)
        if rc != OK:
            raise RuntimeError(f"blsgpu_signing_roots -> {code_name(rc)}")
        return [out[32 * i: 32 * i + 32].tobytes() for i in range(n)]

    def debug_op(self, op: int, inputs: bytes, in_stride: int, out_stride: int):
        n = len(inputs) // in_stride
        inb = np.frombuffer(inputs, dtype=np.uint8).copy()
        out = np.zeros(n * out_stride, dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        rc = self._lib.blsgpu_debug_op(self.h, op, n, inb.ctypes.data, in_stride, out.ctypes.data, out_stride,
                                       st.ctypes.data)
        if rc != OK:
            raise RuntimeError(f"blsgpu_debug_op -> {code_name(rc)}")
        return out.tobytes(), st
