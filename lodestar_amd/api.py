"""Host-side entry points around the C-ABI for the callers on either side of the verifier path, mirroring the
reference's own functions (same names in snake_case, same argument meaning and error behaviour):

* verify_signature_set           state-transition/src/util/signatureSets.ts:24-38 (single: Signature.verify;
                                 aggregate: Signature.verifyAggregate -- FastAggregateVerify over trusted keys)
* fast_aggregate_verify          beacon-node/test/spec/general/bls.ts:117-127 (untrusted keys: KeyValidate;
                                 any error -> False)
* eth_fast_aggregate_verify      beacon-node/test/spec/general/bls.ts:93-112
* eth_aggregate_pubkeys          beacon-node/test/spec/general/bls.ts:75-83 (an infinity key -> None)
* process_deposit_signature      state-transition/src/block/processDeposit.ts:54-64 (KeyValidate + verify;
                                 any error -> False: the deposit is skipped, not rejected)

All of them run on the GPU through lodestar_amd.native.Context (there is no CPU path).
"""
import numpy as np

from lodestar_amd.native import Context, code_name

G1_INFINITY_48 = bytes([0xC0]) + bytes(47)
G2_INFINITY_96 = bytes([0xC0]) + bytes(95)


class BlstError(Exception):
    """Mirrors @chainsafe/blst's ErrorBLST: the message carries 'BLST_ERROR: <CODE>'."""

    def __init__(self, code):
        self.code = code
        name = code_name(code)
        super().__init__(name if code in (9, 10) else f"BLST_ERROR: {name}")


def _one_job(ctx: Context, pk96_list, msg: bytes, sig: bytes):
    """One non-batchable job of one set whose pubkeys (96-byte uncompressed) are aggregated on the GPU."""
    sig = bytes(sig)
    sig_buf = sig.ljust(192, b"\0")[:192]
    res, _ = ctx.verify_raw([0, 1], sig_buf, [len(sig)], bytes(msg)[:32].ljust(32, b"\0"),
                            pk_bytes=b"".join(pk96_list) or bytes(96), set_pk_first=[0, len(pk96_list)],
                            job_flags=[0], sig_stride=192)
    return int(res[0])


def verify_signature_set(ctx: Context, pubkeys96, signing_root: bytes, signature: bytes) -> bool:
    """verifySignatureSet: `pubkeys96` is one trusted key (single set) or a list (aggregate set).  Raises
    BlstError where Signature.fromBytes(validate=true) throws."""
    keys = [pubkeys96] if isinstance(pubkeys96, (bytes, bytearray)) else list(pubkeys96)
    r = _one_job(ctx, keys, signing_root, signature)
    if r < 0:
        raise BlstError(-r)
    return r == 1


def key_validate(ctx: Context, pubkeys48):
    """KeyValidate of 48-byte keys: (list of 96-byte uncompressed or None, status array)."""
    if not pubkeys48:
        return [], np.zeros(0, np.int8)
    if any(len(p) != 48 for p in pubkeys48):
        raise ValueError("48-byte compressed pubkeys expected")
    pk96, st = ctx.key_validate(b"".join(bytes(p) for p in pubkeys48), 48)
    return [pk96[96 * i: 96 * i + 96] if st[i] == 0 else None for i in range(len(pubkeys48))], st


def fast_aggregate_verify(ctx: Context, pubkeys48, message: bytes, signature: bytes) -> bool:
    keys, st = key_validate(ctx, list(pubkeys48))
    if not keys or (st != 0).any():
        return False  # EMPTY_AGGREGATE_ARRAY / BLST_* -> caught -> false
    return _one_job(ctx, keys, message, signature) == 1


def eth_fast_aggregate_verify(ctx: Context, pubkeys48, message: bytes, signature: bytes) -> bool:
    pubkeys48 = [bytes(p) for p in pubkeys48]
    if not pubkeys48 and bytes(signature) == G2_INFINITY_96:
        return True
    if any(p == G1_INFINITY_48 for p in pubkeys48):
        return False
    return fast_aggregate_verify(ctx, pubkeys48, message, signature)


def eth_aggregate_pubkeys(ctx: Context, pubkeys48):
    """Aggregate of untrusted compressed keys -> 48-byte compressed, None where the spec runner returns null."""
    pubkeys48 = [bytes(p) for p in pubkeys48]
    if not pubkeys48 or any(p == G1_INFINITY_48 for p in pubkeys48):
        return None
    keys, st = key_validate(ctx, pubkeys48)
    if (st != 0).any():
        return None
    out, ast = ctx.aggregate_pubkeys(pk_bytes=b"".join(keys), set_pk_first=[0, len(keys)], out_len=48)
    return out[0] if ast[0] == 0 else None


def process_deposit_signature(ctx: Context, pubkey48: bytes, signing_root: bytes, signature: bytes) -> bool:
    """processDeposit's signature check: PublicKey.fromBytes(validate) + Signature.fromBytes(validate) +
    verify, and `catch { return false }` -- an invalid deposit is skipped, never thrown."""
    keys, st = key_validate(ctx, [pubkey48])
    if st[0] != 0:
        return False
    return _one_job(ctx, keys, signing_root, signature) == 1


def process_deposit_signatures(ctx: Context, pubkeys48, signing_roots, signatures):
    """process_deposit_signature over many deposits in two GPU calls (KeyValidate of every key, then one
    non-batchable single-set job per deposit with a valid key): list of bools."""
    n = len(pubkeys48)
    if n == 0:
        return []
    keys, st = key_validate(ctx, [bytes(p) for p in pubkeys48])
    ok = [i for i in range(n) if st[i] == 0]
    out = [False] * n
    if not ok:
        return out
    sigs = [bytes(signatures[i]) for i in ok]
    res, _ = ctx.verify_raw(np.arange(len(ok) + 1), b"".join(s.ljust(192, b"\0")[:192] for s in sigs),
                            [len(s) for s in sigs], b"".join(bytes(signing_roots[i])[:32] for i in ok),
                            pk_bytes=b"".join(keys[i] for i in ok), job_flags=np.zeros(len(ok)), sig_stride=192)
    for k, i in enumerate(ok):
        out[i] = int(res[k]) == 1  # errors (malformed signature) and false both skip the deposit
    return out
