"""The group-by's 128-bit record form of canonical UUID keys (deequ_amd/csrc/dq_uuidpack.h),
through the host build dq_diag_uuid_pack: every canonical lowercase UUID packs to two words that
unpack to the same text, distinct UUIDs get distinct words, and nothing else packs (uppercase,
misplaced or missing dashes, non-hex bytes, other lengths keep the hashed records)."""
import ctypes
import random
import uuid

from deequ_amd import _lib as L


def pack(key: bytes):
    words = (ctypes.c_uint64 * 2)()
    back = ctypes.create_string_buffer(36)
    ok = ctypes.c_int32()
    L.check(L.lib().dq_diag_uuid_pack(key, len(key), words, back, ctypes.byref(ok)))
    if not ok.value:
        return None
    return (words[0], words[1]), back.raw


def test_layout():
    # hex group g of the text -> bits 16 g of lo (g < 4) / hi; byte i of a group -> nibble i
    (lo, hi), back = pack(b"01234567-89ab-cdef-0123-456789abcdef")
    assert back == b"01234567-89ab-cdef-0123-456789abcdef"
    assert lo == 0xFEDC_BA98_7654_3210 and hi == 0xFEDC_BA98_7654_3210
    assert pack(b"00000000-0000-0000-0000-000000000000")[0] == (0, 0)
    assert pack(b"ffffffff-ffff-ffff-ffff-ffffffffffff")[0] == (2 ** 64 - 1, 2 ** 64 - 1)


def test_round_trip_and_distinct():
    rng = random.Random(7)
    seen = {}
    for _ in range(20000):
        u = str(uuid.UUID(int=rng.getrandbits(128))).encode()
        words, back = pack(u)
        assert back == u
        assert seen.setdefault(words, u) == u
    # every value of one hex group position, each character class boundary
    for c in b"0123456789abcdef":
        u = b"0" * 8 + b"-" + bytes([c]) * 4 + b"-0000-0000-" + b"0" * 12
        assert pack(u)[1] == u


def test_not_canonical():
    good = b"01234567-89ab-cdef-0123-456789abcdef"
    assert pack(good.upper()) is None
    assert pack(good[:-1]) is None and pack(good + b"0") is None
    for i in (8, 13, 18, 23):
        assert pack(good[:i] + b"0" + good[i + 1:]) is None  # a dash replaced
    for i in (0, 7, 9, 12, 14, 17, 19, 22, 24, 35):
        for bad in (b"g", b"G", b"/", b":", b"`", b"-", b"\x80", b"\xff", b" "):
            assert pack(good[:i] + bad + good[i + 1:]) is None, (i, bad)
    assert pack(b"") is None
