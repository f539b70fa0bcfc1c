"""The group-by's 8-byte record form of digit-string keys (deequ_amd/csrc/dq_keypack.h), through
the host build dq_diag_key_pack: every key of <= 15 ASCII digits (and Histogram's "NullValue")
packs to a word that unpacks to the same bytes, distinct keys get distinct words, and nothing
else packs (the partition path then stages it as a 16-byte record)."""
import ctypes
import random

import pytest

from deequ_amd import _lib as L


def pack(key: bytes):
    packed = ctypes.c_uint64()
    back = ctypes.create_string_buffer(16)
    back_len = ctypes.c_int32()
    ok = ctypes.c_int32()
    L.check(L.lib().dq_diag_key_pack(key, len(key), ctypes.byref(packed), back, ctypes.byref(back_len),
                                     ctypes.byref(ok)))
    if not ok.value:
        return None
    return packed.value, back.raw[:back_len.value]


def test_layout():
    # nibble i = digit i, length in the top nibble
    assert pack(b"0123") == ((4 << 60) | 0x3210, b"0123")
    assert pack(b"") == (0, b"")
    assert pack(b"9" * 15) == ((15 << 60) | int("9" * 15, 16), b"9" * 15)
    assert pack(b"NullValue") == (0xA, b"NullValue")


def test_round_trip_and_distinct():
    rng = random.Random(5)
    seen = {}
    keys = {b""} | {b"0" * n for n in range(16)} | {("%012d" % v).encode() for v in range(0, 10**12, 10**9 + 7)}
    for _ in range(20000):
        n = rng.randint(0, 15)
        keys.add(bytes(rng.choice(b"0123456789") for _ in range(n)))
    for k in keys:
        r = pack(k)
        assert r is not None, k
        p, back = r
        assert back == k
        assert p not in seen, (k, seen.get(p))
        seen[p] = k
    assert 0xA not in seen and (1 << 64) - 1 not in seen and (1 << 64) - 2 not in seen


@pytest.mark.parametrize("bad", [b"12a4", b"/", b":", b"12 3", b"\x00", b"1\x80", b"\xb0\xb9", b"9" * 16,
                                 b"0" * 16, b"-1", b"+5", b"1.5", b"NullValu", b"nullvalue"])
def test_not_packed(bad):
    assert pack(bad) is None


def test_every_single_byte():
    for b in range(256):
        r = pack(bytes([b]) + b"7")
        assert (r is not None) == (0x30 <= b <= 0x39), b
