"""The group-by's table hash on the device (dq_diag_table_hash) against a host restatement.
Every path (stage, splits, aggregations, inserts, imports, lookups, rehash, owner ranks) places
a key with this one function, so it must be a pure function of the key bytes -- a packed digit
record (deequ_amd/csrc/dq_keypack.h) hashes to the same value as the key it packs: a key
that packs (digits, or "NullValue") is hashed as its packed word, any other with hash_raw."""
import ctypes
import random

import numpy as np
import pytest

from deequ_amd import _lib as L

pytestmark = pytest.mark.gpu
M = (1 << 64) - 1


def hash_raw(k0, k1, n):
    a = ((k0 + 0x165667B19E3779F9) & M) * 0x9E3779B97F4A7C15 & M
    b = ((k1 ^ (n << 56) ^ 0x27D4EB2F165667C5) * 0xC2B2AE3D27D4EB4F) & M
    h = a ^ (((b << 32) | (b >> 32)) & M)
    h ^= h >> 29
    h = (h * 0xD6E8FEB86659FD93) & M
    return h ^ (h >> 32)


def hash_packed(p):
    x = (p + 0x9E3779B97F4A7C15) & M
    x ^= x >> 32
    x = (x * 0xD6E8FEB86659FD93) & M
    x ^= x >> 32
    x = (x * 0xD6E8FEB86659FD93) & M
    return x ^ (x >> 32)


def pack(key: bytes):
    if len(key) <= 15 and all(0x30 <= c <= 0x39 for c in key):
        p = len(key) << 60
        for i, c in enumerate(key):
            p |= (c - 0x30) << (4 * i)
        return p
    return None


def expect(key: bytes):
    k = key.ljust(16, b"\0")
    k0, k1 = int.from_bytes(k[:8], "little"), int.from_bytes(k[8:], "little")
    p = pack(key)
    rec = p if p is not None else (0xA if key == b"NullValue" else M)
    h = hash_packed(rec) if rec != M else hash_raw(k0, k1, len(key))
    return k0, k1, h, rec


def test_table_hash_matches_host(gpu):
    rng = random.Random(9)
    keys = [int(v).to_bytes(8, "little", signed=True) for v in list(range(0, 300_000, 13)) + [987_654_321, -1, -2**63]]
    keys += [("%012d" % rng.randrange(10**12)).encode() for _ in range(20000)]
    keys += [bytes(rng.choice(b"0123456789") for _ in range(rng.randint(0, 15))) for _ in range(5000)]
    keys += [bytes(rng.randrange(256) for _ in range(rng.randint(0, 16))) for _ in range(5000)]
    keys += [b"NullValue", b"", b"0", b"00", b"0" * 15, b"0" * 16, b"k12", b"9" * 15]
    want = [expect(k) for k in keys]
    k0 = np.array([w[0] for w in want], dtype=np.uint64)
    k1 = np.array([w[1] for w in want], dtype=np.uint64)
    ln = np.array([len(k) for k in keys], dtype=np.uint32)
    out = np.zeros(2 * len(keys), dtype=np.uint64)
    L.check(L.lib().dq_diag_table_hash(0, k0.ctypes.data, k1.ctypes.data, ln.ctypes.data, len(keys), out.ctypes.data))
    bad = [(k, hex(int(out[2 * i])), hex(w[2]), hex(int(out[2 * i + 1])), hex(w[3]))
           for i, (k, w) in enumerate(zip(keys, want)) if int(out[2 * i]) != w[2] or int(out[2 * i + 1]) != w[3]]
    assert not bad, (len(bad), bad[:5])
