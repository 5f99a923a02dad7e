"""Minimal SSZ hash_tree_root helpers for building reference known-answer inputs -- TEST
INFRASTRUCTURE ONLY (consensus-specs phase0 `compute_signing_root`, `compute_domain`; reference
`packages/state-transition/src/util/signingRoot.ts:7-13`, `util/domain.ts`)."""
import hashlib


def _h(a, b):
    return hashlib.sha256(a + b).digest()


def merkleize(chunks):
    n = 1
    while n < len(chunks):
        n *= 2
    layer = list(chunks) + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [_h(layer[i], layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def bytes_root(b):
    chunks = [b[i:i + 32].ljust(32, b"\x00") for i in range(0, len(b), 32)]
    return merkleize(chunks)


def uint64_root(v):
    return v.to_bytes(8, "little").ljust(32, b"\x00")


def deposit_message_root(pubkey, withdrawal_credentials, amount):
    return merkleize([bytes_root(pubkey), bytes_root(withdrawal_credentials), uint64_root(amount)])


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes = bytes(32)):
    fork_data_root = merkleize([bytes_root(fork_version), genesis_validators_root])
    return domain_type + fork_data_root[:28]


def compute_signing_root(object_root: bytes, domain: bytes):
    return merkleize([object_root, domain])


DOMAIN_DEPOSIT = bytes.fromhex("03000000")
