"""Java hashCode of a stored value, as DistinctCountBitmapAggregationFunction.java adds it to its RoaringBitmap
(convertToValueBitmap, :410-446): INT the value, LONG Long.hashCode, FLOAT Float.hashCode (floatToIntBits), DOUBLE
Double.hashCode, STRING String.hashCode over UTF-16 code units. Signed 32-bit results (the bitmap treats them as
unsigned ints: the distinct count is the same)."""
import struct

_M32 = 0xFFFFFFFF


def _s32(x):
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def java_hash_code(value, data_type):
    if data_type == "INT":
        return _s32(int(value))
    if data_type == "LONG":
        v = int(value) & 0xFFFFFFFFFFFFFFFF
        return _s32(v ^ (v >> 32))
    if data_type == "FLOAT":
        f = float(value)
        if f != f:
            return _s32(0x7FC00000)  # floatToIntBits: the canonical NaN
        return _s32(struct.unpack(">I", struct.pack(">f", f))[0])
    if data_type == "DOUBLE":
        d = float(value)
        bits = 0x7FF8000000000000 if d != d else struct.unpack(">Q", struct.pack(">d", d))[0]
        return _s32(bits ^ (bits >> 32))
    if data_type == "STRING":
        h = 0
        units = str(value).encode("utf-16-be")
        for i in range(0, len(units), 2):
            h = (31 * h + ((units[i] << 8) | units[i + 1])) & _M32
        return _s32(h)
    raise ValueError("DISTINCTCOUNTBITMAP: unsupported data type %s" % data_type)
