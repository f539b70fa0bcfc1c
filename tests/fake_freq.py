"""Host stand-in for deequ_amd.frequencies.FrequencyTable, used ONLY by the CPU (gloo) tests of
the multi-rank exchange orchestration (deequ_amd/distributed.py): same methods, same wire layout
(per part: 16-B packed records for keys that pack into one word, then 32-B general records),
groups kept in a dict.  The GPU tests run the same orchestration on the real table."""
import struct
from typing import Dict, List, Tuple

import numpy as np
import torch

from deequ_amd.frequencies import FrequencyTable, encode_key

HEAP = 1 << 30


PACK_NULL = 0xA


def pack(key: bytes):
    """dq_keypack.h: a digit string of <= 15 bytes (nibble i = digit i, length in the top nibble),
    Histogram's "NullValue" as PACK_NULL; None for any other key."""
    if key == b"NullValue":
        return PACK_NULL
    if len(key) > 15 or not all(0x30 <= c <= 0x39 for c in key):
        return None
    p = len(key) << 60
    for i, c in enumerate(key):
        p |= (c - 0x30) << (4 * i)
    return p


def unpack(p: int) -> bytes:
    if p == PACK_NULL:
        return b"NullValue"
    n = p >> 60
    return bytes(0x30 + ((p >> (4 * i)) & 0xF) for i in range(n))


class FakeFrequencyTable:
    WIRE_PACKED_BYTES = 16
    WIRE_BYTES = 32

    @classmethod
    def part_bytes(cls, packed, general):
        return cls.WIRE_PACKED_BYTES * int(packed) + cls.WIRE_BYTES * int(general)

    def __init__(self, key_columns, schema, histogram=False, device=None):
        self.key_columns = list(key_columns)
        self.schema = dict(schema)
        self.dtypes = [self.schema[c] for c in self.key_columns]
        self.histogram = histogram
        self.groups: Dict[bytes, int] = {}
        self.num_rows = 0

    @classmethod
    def like(cls, other):
        return cls(other.key_columns, {c: t for c, t in zip(other.key_columns, other.dtypes)}, other.histogram)

    @property
    def torch_device(self):
        return torch.device("cpu")

    def consume(self, batch):
        cols = [batch.columns[c].to_pylist() for c in self.key_columns]
        for row in zip(*cols):
            self.num_rows += 1
            if not self.histogram and any(v is None for v in row):
                continue
            k = encode_key(row, self.dtypes, self.histogram)
            self.groups[k] = self.groups.get(k, 0) + 1

    def summary(self):
        class S:
            pass
        s = S()
        s.num_rows = self.num_rows
        return s

    @staticmethod
    def _owner(key: bytes, n: int) -> int:
        return (sum(key) * 2654435761 + len(key)) % n

    def _parts(self, n):
        parts = [[] for _ in range(n)]
        for k in sorted(self.groups):
            parts[self._owner(k, n)].append(k)
        return parts

    def partition_sizes(self, n) -> Tuple[List[int], List[int], List[int]]:
        parts = self._parts(n)
        packed = [sum(1 for k in p if pack(k) is not None) for p in parts]
        general = [len(p) - c for p, c in zip(parts, packed)]
        kb = [sum((len(k) + 7) // 8 * 8 for k in p if len(k) > 16 and pack(k) is None) for p in parts]
        return packed, general, kb

    def partition_into(self, n, groups, keys):
        g = groups.numpy()
        kb = keys.numpy()
        go, ko = 0, 0
        for p in self._parts(n):
            base = ko
            for k in [k for k in p if pack(k) is not None]:
                g[go:go + 16] = np.frombuffer(struct.pack("<Qq", pack(k), self.groups[k]), dtype=np.uint8)
                go += 16
            for k in [k for k in p if pack(k) is None]:
                if len(k) <= 16:
                    pad = k + b"\0" * (16 - len(k))
                    rec = struct.pack("<Qq", len(k), self.groups[k]) + pad
                else:
                    off = ko - base
                    kb[ko:ko + len(k)] = np.frombuffer(k, dtype=np.uint8)
                    ko += (len(k) + 7) // 8 * 8
                    rec = struct.pack("<QqQQ", HEAP | len(k), self.groups[k], off, 0)
                g[go:go + 32] = np.frombuffer(rec, dtype=np.uint8)
                go += 32
        return self.partition_sizes(n)

    def import_parts(self, parts, packed, general, keys, key_bytes, num_rows=0):
        g = bytes(parts.numpy())
        kb = bytes(keys.numpy())
        self.num_rows += num_rows
        go, ko = 0, 0
        for np_, ng, nk in zip(packed, general, key_bytes):
            for i in range(np_):
                p, cnt = struct.unpack_from("<Qq", g, go + 16 * i)
                k = unpack(p)
                self.groups[k] = self.groups.get(k, 0) + cnt
            go += 16 * np_
            self._import_general(g[go:go + 32 * ng], ng, kb[ko:ko + nk])
            go += 32 * ng
            ko += nk

    def import_wire(self, groups, n, keys, key_bytes, num_rows=0):
        self.num_rows += num_rows
        self._import_general(bytes(groups.numpy()[:n * 32]), n, bytes(keys.numpy()[:key_bytes]))

    def _import_general(self, g, n, kb):
        for i in range(n):
            ctrl, cnt, k0, k1 = struct.unpack_from("<QqQQ", g, i * 32)
            ln = ctrl & ((1 << 24) - 1)
            if ctrl & HEAP:
                k = kb[k0:k0 + ln]
            else:
                k = (struct.pack("<QQ", k0, k1))[:ln]
            self.groups[k] = self.groups.get(k, 0) + cnt

    def count_histogram(self, n_bins=1 << 16):
        hist = np.zeros(n_bins, dtype=np.int64)
        big = []
        for c in self.groups.values():
            if c < n_bins:
                hist[c] += 1
            else:
                big.append(c)
        return hist, np.array(sorted(big), dtype=np.int64)

    def top(self, n):
        items = sorted(self.groups.items(), key=lambda kv: (-kv[1], kv[0]))
        if len(items) > n:
            cut = items[n - 1][1]
            items = [kv for kv in items if kv[1] >= cut]
        return np.array([c for _, c in items], dtype=np.int64), [k for k, _ in items]

    def export(self):
        return np.array(list(self.groups.values()), dtype=np.int64), list(self.groups.keys())

    to_arrow = FrequencyTable.to_arrow  # (built on export_flat only)

    def export_flat(self, device=False):
        counts, keys = self.export()
        offs = np.zeros(len(keys) + 1, dtype=np.int64)
        np.cumsum([len(k) for k in keys], out=offs[1:])
        return counts, offs, np.frombuffer(b"".join(keys), dtype=np.uint8).copy()

    def close(self):
        pass
