"""TEST INFRASTRUCTURE ONLY: oracle-signed signature sets with ~1% of the sets corrupted in every way the
reference distinguishes, for the GPU parity tests (tests/) and bench.py's untimed parity leg.

Only tests/, __graft_entry__ and bench.py's checker legs (cpu_baseline, parity) import this module; the product
(lodestar_amd) never does.  The classes follow the reference's contract (SURVEY.md 8a A8 / parity contract):
  * a well-formed signature over another message, another set's signature, the negated signature, and the
    identity (compressed 0xc0.. or uncompressed 0x40..) -> the set fails the pairing equation (job `false`);
  * Signature.fromBytes(sig, affine, validate=true) errors (maybeBatch.ts:23,36) -> the job throws:
    BLST_INVALID_SIZE (48- or 0-byte signature, multithread.test.ts:100), BLST_BAD_ENCODING (x >= p, compression
    flag cleared on 96 B, set on 192 B), BLST_POINT_NOT_ON_CURVE (compressed x with no y; an uncompressed point
    with y moved), BLST_POINT_NOT_IN_GROUP (a curve point outside G2);
  * a valid signature re-encoded uncompressed (192 B) -> still valid.
"""
import functools
import hashlib

import numpy as np

from . import bls12_381 as bls
from . import cpu

# kind -> what the reference does with the set's job (for the report; the oracle gives the actual value)
KINDS = ["wrong_msg", "swap", "negated", "infinity", "infinity_192", "size_48", "size_0", "bad_flag_96",
         "x_ge_p", "flag_on_192", "not_on_curve", "not_on_curve_192", "not_in_group", "uncompressed_valid"]


@functools.lru_cache(maxsize=1)
def adversarial_sigs():
    """One compressed signature per fromBytes decode class, the first candidates of a fixed scan (classified by
    the C oracle, cross-checked with the Python oracle)."""
    out = {}
    for t in range(1, 4000):
        cand = bytes([0x80]) + bytes(45) + t.to_bytes(2, "big") + bytes(48)
        c = cpu.sig_status(cand)
        if c in (bls.BLST_POINT_NOT_ON_CURVE, bls.BLST_POINT_NOT_IN_GROUP) and c not in out:
            assert bls.classify_signature(cand) == c
            out[c] = cand
        if len(out) == 2:
            break
    return out


def _uncompressed(sig96):
    return bls.g2_serialize(bls.signature_from_bytes(sig96, validate=False))


def corrupt_sets(sigs96, msgs, rng, frac=0.01, min_bad=len(KINDS), kinds=KINDS):
    """Corrupts ~frac of the sets (at least min_bad), cycling through `kinds`.

    sigs96: list of 96-byte valid signatures, msgs: list of 32-byte signing roots (set i signs msgs[i]).
    Returns (msgs, sig_buf with a 192-byte stride, sig_len list, {set index: kind})."""
    n = len(sigs96)
    msgs = list(msgs)
    sig_list = list(sigs96)
    sig_len = [96] * n
    n_bad = min(n, max(min_bad, int(round(n * frac))))
    bad = sorted(rng.choice(n, size=n_bad, replace=False).tolist())
    adv = adversarial_sigs()
    applied = {}
    for k, i in enumerate(bad):
        kind = kinds[k % len(kinds)]
        s = sig_list[i]
        if kind == "wrong_msg":
            msgs[i] = hashlib.sha256(b"another message" + msgs[i]).digest()
        elif kind == "swap":
            sig_list[i] = sigs96[(i + 1) % n]
        elif kind == "negated":
            sig_list[i] = bytes([s[0] ^ 0x20]) + s[1:]  # sort flag flipped: -sig, a valid G2 point
        elif kind == "infinity":
            sig_list[i] = bytes([0xC0]) + bytes(95)
        elif kind == "infinity_192":
            sig_list[i] = bytes([0x40]) + bytes(191)
            sig_len[i] = 192
        elif kind == "size_48":
            sig_list[i] = s[:48]
            sig_len[i] = 48
        elif kind == "size_0":
            sig_list[i] = b""
            sig_len[i] = 0
        elif kind == "bad_flag_96":
            sig_list[i] = bytes([s[0] & 0x7F]) + s[1:]
        elif kind == "x_ge_p":
            sig_list[i] = bytes([0x80 | 0x1F]) + bytes([0xFF]) * 95
        elif kind == "flag_on_192":
            u = _uncompressed(s)
            sig_list[i] = bytes([u[0] | 0x80]) + u[1:]
            sig_len[i] = 192
        elif kind == "not_on_curve":
            sig_list[i] = adv[bls.BLST_POINT_NOT_ON_CURVE]
        elif kind == "not_on_curve_192":
            u = bytearray(_uncompressed(s))
            u[191] ^= 1
            sig_list[i] = bytes(u)
            sig_len[i] = 192
        elif kind == "not_in_group":
            sig_list[i] = adv[bls.BLST_POINT_NOT_IN_GROUP]
        elif kind == "uncompressed_valid":
            sig_list[i] = _uncompressed(s)
            sig_len[i] = 192
        else:
            raise ValueError(kind)
        applied[i] = kind
    sig_buf = b"".join(x.ljust(192, b"\0") for x in sig_list)
    return msgs, sig_buf, sig_len, applied


def result_classes(results):
    """Histogram of per-job results by name (1 valid, 0 false, -code -> the BLST code name)."""
    names = {1: "valid", 0: "false", -bls.BLST_BAD_ENCODING: "BLST_BAD_ENCODING",
             -bls.BLST_POINT_NOT_ON_CURVE: "BLST_POINT_NOT_ON_CURVE",
             -bls.BLST_POINT_NOT_IN_GROUP: "BLST_POINT_NOT_IN_GROUP", -bls.BLST_INVALID_SIZE: "BLST_INVALID_SIZE",
             -bls.BLST_PK_IS_INFINITY: "BLST_PK_IS_INFINITY", -9: "EMPTY_AGGREGATE_ARRAY", -10: "Empty signature set"}
    vals, counts = np.unique(np.asarray(results, np.int64), return_counts=True)
    return {names.get(int(v), f"code_{int(v)}"): int(c) for v, c in zip(vals, counts)}
