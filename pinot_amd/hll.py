"""HyperLogLog intermediate result (the DISTINCTCOUNTHLL DataTable value), host side.

The reference uses com.clearspring.analytics:stream 2.9.8 (pom.xml:1184-1186, not vendored in the
reference). Its published algorithm, restated here for the values the GPU registers feed:
  * MurmurHash.hash(Object): Integer/Long -> hashLong(v); Float -> hashLong(floatToRawIntBits(v));
    Double -> hashLong(doubleToRawLongBits(v)); String -> hash(getBytes(UTF-8), length, seed=-1).
  * offerHashed(h): j = h >>> (32 - log2m); r = numberOfLeadingZeros((h << log2m) | (1 << (log2m-1)) + 1) + 1;
    register[j] = max(register[j], r).
  * cardinality(): registerSum = sum 1/(1 << reg); estimate = alphaMM / registerSum;
    estimate <= 2.5*m ? round(m * ln(m / zeros)) : round(estimate).
  * getBytes(): big-endian int log2m, int (RegisterSet.size*4), then the RegisterSet words (5-bit registers
    packed 6 per 32-bit word, LOG2_BITS_PER_WORD=6, REGISTER_SIZE=5).
Pinned by the reference's golden cardinalities (InterSegmentAggregationSingleValueQueriesTest.java:261-283).
"""
import math
import struct

import numpy as np

_M32 = 0xFFFFFFFF


def _i32(x):
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def hash_long(data: int) -> int:
    """MurmurHash.hashLong(long) (32-bit result, signed)."""
    m = 0x5BD1E995
    r = 24
    h = 0
    k = (data & _M32) * m & _M32
    k ^= k >> r
    h ^= k * m & _M32
    k = ((data >> 32) & _M32) * m & _M32
    k ^= k >> r
    h = h * m & _M32
    h ^= k * m & _M32
    h ^= h >> 13
    h = h * m & _M32
    h ^= h >> 15
    return _i32(h)


def hash_bytes(data: bytes, seed: int = -1) -> int:
    """MurmurHash.hash(byte[], length, seed) — MurmurHash2, Java signed-byte semantics."""
    m = 0x5BD1E995
    length = len(data)
    h = (seed ^ length) & _M32
    n4 = length >> 2
    sb = [b - 256 if b > 127 else b for b in data]
    for i in range(n4):
        i4 = i << 2
        k = sb[i4 + 3]
        k = (k << 8) | (data[i4 + 2])
        k = (k << 8) | (data[i4 + 1])
        k = (k << 8) | (data[i4 + 0])
        k &= _M32
        k = k * m & _M32
        k ^= k >> 24
        k = k * m & _M32
        h = h * m & _M32
        h ^= k
    left = length - (n4 << 2)
    if left:
        if left >= 3:
            h ^= (sb[length - 3] << 16) & _M32
        if left >= 2:
            h ^= (sb[length - 2] << 8) & _M32
        if left >= 1:
            h ^= sb[length - 1] & _M32
        h = h * m & _M32
    h ^= h >> 13
    h = h * m & _M32
    h ^= h >> 15
    return _i32(h)


def hash_value(value, data_type: str) -> int:
    """MurmurHash.hash(Object) for the boxed value a Pinot Dictionary returns for the column type."""
    if data_type in ("INT", "LONG"):
        return hash_long(int(value))
    if data_type == "FLOAT":
        bits = struct.unpack("<i", struct.pack("<f", float(value)))[0]
        return hash_long(bits)
    if data_type == "DOUBLE":
        bits = struct.unpack("<q", struct.pack("<d", float(value)))[0]
        return hash_long(bits)
    if data_type == "STRING":
        return hash_bytes(str(value).encode("utf-8"))
    raise ValueError("unsupported type " + data_type)


def slot_rank(hashed: int, log2m: int):
    h = hashed & _M32
    j = h >> (32 - log2m)
    x = ((h << log2m) & _M32) | ((1 << (log2m - 1)) + 1)
    r = (32 - x.bit_length()) + 1
    return j, r


def register_set_words(m: int) -> int:
    """RegisterSet.getSizeForCount."""
    bits = m // 6
    if bits == 0:
        return 1
    return bits if bits % 32 == 0 else bits + 1


class HyperLogLog:
    def __init__(self, log2m=8, registers=None):
        self.log2m = int(log2m)
        m = 1 << self.log2m
        self.registers = np.zeros(m, dtype=np.uint8) if registers is None else np.asarray(registers, dtype=np.uint8).copy()
        assert self.registers.shape == (m,)

    def offer_hashed(self, hashed: int):
        j, r = slot_rank(hashed, self.log2m)
        if r > self.registers[j]:
            self.registers[j] = r

    def offer(self, value, data_type):
        self.offer_hashed(hash_value(value, data_type))

    def add_all(self, other: "HyperLogLog"):
        if other.log2m != self.log2m:
            raise ValueError("Cannot merge estimators of different sizes")
        np.maximum(self.registers, other.registers, out=self.registers)
        return self

    def cardinality(self) -> int:
        m = 1 << self.log2m
        register_sum = 0.0
        zeros = 0.0
        for v in self.registers.tolist():
            register_sum += 1.0 / (1 << v)
            if v == 0:
                zeros += 1
        if self.log2m == 4:
            alpha_mm = 0.673 * m * m
        elif self.log2m == 5:
            alpha_mm = 0.697 * m * m
        elif self.log2m == 6:
            alpha_mm = 0.709 * m * m
        else:
            alpha_mm = (0.7213 / (1 + 1.079 / m)) * m * m
        estimate = alpha_mm * (1 / register_sum)
        if estimate <= (5.0 / 2.0) * m:
            if zeros == 0:
                # linearCounting(m, 0.0) = m * log(m / 0.0) = +Infinity; Math.round(+Infinity) == Long.MAX_VALUE
                return (1 << 63) - 1
            return int(math.floor(m * math.log(m / zeros) + 0.5))  # Math.round
        return int(math.floor(estimate + 0.5))

    def to_bytes(self) -> bytes:
        m = 1 << self.log2m
        words = [0] * register_set_words(m)
        for pos, v in enumerate(self.registers.tolist()):
            b = pos // 6
            shift = 5 * (pos - b * 6)
            words[b] |= (v & 0x1F) << shift
        out = struct.pack(">ii", self.log2m, len(words) * 4)
        return out + b"".join(struct.pack(">I", w & _M32) for w in words)

    @classmethod
    def from_bytes(cls, b: bytes) -> "HyperLogLog":
        log2m, nbytes = struct.unpack_from(">ii", b, 0)
        words = struct.unpack_from(">%dI" % (nbytes // 4), b, 8)
        m = 1 << log2m
        regs = np.zeros(m, dtype=np.uint8)
        for pos in range(m):
            bb = pos // 6
            regs[pos] = (words[bb] >> (5 * (pos - bb * 6))) & 0x1F
        return cls(log2m, regs)

    def __eq__(self, other):
        return isinstance(other, HyperLogLog) and self.log2m == other.log2m and \
            np.array_equal(self.registers, other.registers)

    def __repr__(self):
        return "HyperLogLog(log2m=%d, cardinality=%d)" % (self.log2m, self.cardinality())
