"""Minimal Avro object-container reader (null/deflate codecs, records of primitive/union fields).

Test infrastructure only: used by make_golden.py to turn the reference's own test input
(pinot-core/src/test/resources/data/test_data-sv.avro) into a committed numpy fixture.
"""
import json
import zlib


def _read_long(buf, pos):
    shift = 0
    acc = 0
    while True:
        b = buf[pos]
        pos += 1
        acc |= (b & 0x7F) << shift
        if not (b & 0x80):
            break
        shift += 7
    return (acc >> 1) ^ -(acc & 1), pos


def _read_bytes(buf, pos):
    n, pos = _read_long(buf, pos)
    return buf[pos:pos + n], pos + n


def _decode(schema, buf, pos):
    if isinstance(schema, list):
        idx, pos = _read_long(buf, pos)
        return _decode(schema[idx], buf, pos)
    if isinstance(schema, dict):
        t = schema["type"]
        if t == "record":
            out = {}
            for f in schema["fields"]:
                out[f["name"]], pos = _decode(f["type"], buf, pos)
            return out, pos
        if t == "array":
            items = []
            while True:
                n, pos = _read_long(buf, pos)
                if n == 0:
                    break
                if n < 0:
                    n = -n
                    _, pos = _read_long(buf, pos)
                for _ in range(n):
                    v, pos = _decode(schema["items"], buf, pos)
                    items.append(v)
            return items, pos
        return _decode(t, buf, pos)
    if schema == "null":
        return None, pos
    if schema in ("int", "long"):
        return _read_long(buf, pos)
    if schema == "string":
        b, pos = _read_bytes(buf, pos)
        return b.decode("utf-8"), pos
    if schema == "bytes":
        return _read_bytes(buf, pos)
    if schema == "boolean":
        return buf[pos] != 0, pos + 1
    if schema == "float":
        import struct
        return struct.unpack_from("<f", buf, pos)[0], pos + 4
    if schema == "double":
        import struct
        return struct.unpack_from("<d", buf, pos)[0], pos + 8
    raise ValueError("unsupported avro type %r" % (schema,))


def read_avro(path):
    buf = open(path, "rb").read()
    assert buf[:4] == b"Obj\x01", "not an avro container"
    pos = 4
    meta = {}
    while True:
        n, pos = _read_long(buf, pos)
        if n == 0:
            break
        if n < 0:
            n = -n
            _, pos = _read_long(buf, pos)
        for _ in range(n):
            k, pos = _read_bytes(buf, pos)
            v, pos = _read_bytes(buf, pos)
            meta[k.decode()] = v
    sync = buf[pos:pos + 16]
    pos += 16
    schema = json.loads(meta["avro.schema"])
    codec = meta.get("avro.codec", b"null").decode()
    records = []
    while pos < len(buf):
        count, pos = _read_long(buf, pos)
        size, pos = _read_long(buf, pos)
        block = buf[pos:pos + size]
        pos += size
        assert buf[pos:pos + 16] == sync
        pos += 16
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec != "null":
            raise ValueError("codec " + codec)
        bp = 0
        for _ in range(count):
            rec, bp = _decode(schema, block, bp)
            records.append(rec)
    return schema, records
