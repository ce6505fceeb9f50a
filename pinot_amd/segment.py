"""Immutable segment model + creator for the columns the hot path reads.

Mirrors the parts of SegmentIndexCreationDriverImpl the scan path depends on:
  * dictionary: sorted unique values (pinot-segment-local/.../creator/impl/SegmentDictionaryCreator.java),
  * dictionary-encoded SV forward index: FixedBitSVForwardIndexWriter bytes, i.e. PinotDataBitSet.writeInt
    layout (pinot-segment-local/.../io/util/PinotDataBitSet.java:143) — value i at stream bits
    [i*nb, (i+1)*nb), MSB-first, nb = PinotDataBitSet.getNumBitsPerValue(cardinality - 1) (:61),
  * dictionary-encoded MV forward index: FixedBitMVForwardIndexWriter bytes
    (pinot-segment-local/.../creator/impl/fwd/FixedBitMVForwardIndexWriter.java:70-140): big-endian int32 chunk
    offsets | row-start bitmap (one bit per value, MSB-first) | the dictIds of all rows bit-packed back to back,
  * raw (no-dictionary) SV columns: the decoded fixed-width values.
"""
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

NUMERIC_TYPES = ("INT", "LONG", "FLOAT", "DOUBLE")
_NP = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


def num_bits_per_value(max_value: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:61): at least one bit."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()


def pack_bits(ids: np.ndarray, nb: int, chunk: int = 1 << 20) -> np.ndarray:
    """Big-endian (MSB-first) bit packing of non-negative ids < 2**nb; PinotDataBitSet.writeInt layout."""
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    n = ids.shape[0]
    nbytes = (n * nb + 7) // 8
    out = np.zeros(nbytes, dtype=np.uint8)
    shifts = np.arange(nb - 1, -1, -1, dtype=np.uint32)
    chunk -= chunk % 8  # chunk boundaries stay byte aligned
    for s in range(0, n, chunk):
        part = ids[s:s + chunk]
        bits = ((part[:, None] >> shifts) & 1).astype(np.uint8).reshape(-1)
        packed = np.packbits(bits)
        b0 = s * nb // 8
        out[b0:b0 + packed.shape[0]] = packed[: nbytes - b0]
    return out


def unpack_bits(buf: np.ndarray, n: int, nb: int) -> np.ndarray:
    """Vectorised inverse of pack_bits (test helper; the oracle has its own scalar restatement)."""
    bits = np.unpackbits(np.asarray(buf, dtype=np.uint8))[: n * nb].reshape(n, nb).astype(np.uint32)
    w = (1 << np.arange(nb - 1, -1, -1, dtype=np.uint64)).astype(np.uint32)
    return (bits * w).sum(axis=1).astype(np.int32)


@dataclass
class Column:
    name: str
    data_type: str                       # INT LONG FLOAT DOUBLE STRING
    has_dictionary: bool = True
    cardinality: int = 0
    num_bits: int = 0
    dictionary: Optional[np.ndarray] = None   # sorted unique values
    fwd_bytes: Optional[np.ndarray] = None    # uint8, FixedBitSVForwardIndexWriter layout
    raw_values: Optional[np.ndarray] = None   # no-dictionary columns
    is_sorted: bool = False
    single_value: bool = True
    inverted_index: bool = False              # index metadata the filter-statistics restatement needs (the GPU
    range_index: bool = False                 # scan itself never uses an index: filter_stats.py)
    range_index_exact: bool = True            # bit-sliced (v2) range index: exact matches; v1: partial matches
    total_num_values: int = 0                 # MV: values over all docs (FixedBitMVForwardIndexWriter totalNumValues)
    max_num_multi_values: int = 0             # MV: longest row

    def mv_layout(self, num_docs):
        """MV forward index sections: (docs per chunk, chunk-offset bytes, bitmap offset, raw-data offset)."""
        dpc, nchunks = mv_docs_per_chunk(num_docs, self.total_num_values)
        header = nchunks * 4
        bitmap = (self.total_num_values + 7) // 8
        return dpc, header, header, header + bitmap

    def mv_lengths(self, num_docs):
        """Values per doc of a multi-value column (from the forward index's doc-start bitmap)."""
        _, _, boff, roff = self.mv_layout(num_docs)
        starts = np.flatnonzero(np.unpackbits(self.fwd_bytes[boff:roff])[:self.total_num_values])
        return np.diff(np.append(starts, self.total_num_values))

    def mv_dict_ids(self, num_docs):
        """Per-doc dictId arrays decoded from the MV forward index bytes (vectorised test helper)."""
        _, _, boff, roff = self.mv_layout(num_docs)
        tv = self.total_num_values
        starts = np.flatnonzero(np.unpackbits(self.fwd_bytes[boff:roff])[:tv])
        ids = unpack_bits(self.fwd_bytes[roff:], tv, self.num_bits)
        return np.split(ids, starts[1:])

    @property
    def is_numeric(self):
        return self.data_type in NUMERIC_TYPES

    def index_of(self, value) -> int:
        """Dictionary.indexOf: dictId of value, or -1 (sorted dictionaries use binary search)."""
        i = self.insertion_index_of(value)
        return i if i >= 0 else -1

    def insertion_index_of(self, value) -> int:
        """Dictionary.insertionIndexOf: index if present, else -(insertionPoint + 1)."""
        d = self.dictionary
        i = int(np.searchsorted(d, value, side="left"))
        if i < len(d) and d[i] == value:
            return i
        return -(i + 1)


@dataclass
class Segment:
    name: str
    num_docs: int
    columns: Dict[str, Column] = field(default_factory=dict)

    def column(self, name) -> Column:
        if name not in self.columns:
            raise KeyError("column %r not in segment %s" % (name, self.name))
        return self.columns[name]


def _coerce(values, data_type):
    if data_type == "STRING":
        return np.asarray(values).astype(str)
    return np.asarray(values, dtype=_NP[data_type])


def mv_docs_per_chunk(num_docs, total_num_values):
    """FixedBitMVForwardIndexWriter.java:72-74: averageValuesPerDoc = totalNumValues / numDocs (int division, widened to
    float), docsPerChunk = (int) Math.ceil(2048 / averageValuesPerDoc) in float arithmetic; returns (docsPerChunk, numChunks)."""
    if num_docs == 0:
        return 1, 0
    avg = np.float32(total_num_values // num_docs)
    dpc = int(np.ceil(np.float64(np.float32(2048) / avg)))
    return dpc, (num_docs + dpc - 1) // dpc


def write_mv_forward_index(ids_per_doc, num_bits) -> np.ndarray:
    """FixedBitMVForwardIndexWriter byte layout for per-doc dictId arrays (every row holds >= 1 value)."""
    n = len(ids_per_doc)
    lengths = np.array([len(x) for x in ids_per_doc], dtype=np.int64)
    if n and lengths.min() < 1:
        raise ValueError("every multi-value row must hold at least one value (Pinot stores the default null value)")
    total = int(lengths.sum())
    dpc, nchunks = mv_docs_per_chunk(n, total)
    starts = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.int64) if n else np.zeros(0, np.int64)
    header = starts[::dpc][:nchunks].astype(">i4").tobytes()
    bits = np.zeros(((total + 7) // 8) * 8, dtype=np.uint8)
    bits[starts] = 1
    bitmap = np.packbits(bits)
    flat = np.concatenate(ids_per_doc).astype(np.uint32) if n else np.zeros(0, np.uint32)
    raw = pack_bits(flat, num_bits)
    return np.concatenate([np.frombuffer(header, dtype=np.uint8), bitmap, raw]).astype(np.uint8)


def mv_column_from_flat(name, lengths, flat_ids, dictionary, data_type) -> Column:
    """MV column from row lengths + the flat dictId stream (vectorised; synthetic benchmark segments)."""
    lengths = np.asarray(lengths, dtype=np.int64)
    if len(lengths) and lengths.min() < 1:
        raise ValueError("every multi-value row must hold at least one value")
    col = Column(name=name, data_type=data_type, single_value=False)
    col.dictionary = np.asarray(dictionary)
    col.cardinality = int(len(dictionary))
    col.num_bits = num_bits_per_value(max(col.cardinality - 1, 0))
    n = len(lengths)
    total = int(lengths.sum())
    col.total_num_values = total
    col.max_num_multi_values = int(lengths.max()) if n else 0
    dpc, nchunks = mv_docs_per_chunk(n, total)
    starts = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(lengths[:-1], out=starts[1:])
    header = starts[::dpc][:nchunks].astype(">i4").tobytes()
    bits = np.zeros(((total + 7) // 8) * 8, dtype=np.uint8)
    bits[starts] = 1
    col.fwd_bytes = np.concatenate([np.frombuffer(header, dtype=np.uint8), np.packbits(bits),
                                    pack_bits(np.asarray(flat_ids, dtype=np.uint32), col.num_bits)]).astype(np.uint8)
    return col


def build_mv_column(name, rows, data_type) -> Column:
    """Dictionary-encoded multi-value column from per-doc value arrays."""
    rows = [_coerce(np.atleast_1d(r), data_type) for r in rows]
    col = Column(name=name, data_type=data_type, single_value=False)
    flat = np.concatenate(rows) if rows else _coerce([], data_type)
    dictionary = np.unique(flat)
    col.dictionary = dictionary
    col.cardinality = int(len(dictionary))
    col.num_bits = num_bits_per_value(max(col.cardinality - 1, 0))
    ids = [np.searchsorted(dictionary, r).astype(np.uint32) for r in rows]
    col.total_num_values = int(len(flat))
    col.max_num_multi_values = int(max((len(r) for r in rows), default=0))
    col.fwd_bytes = write_mv_forward_index(ids, col.num_bits)
    return col


def build_column(name, values, data_type, has_dictionary=True) -> Column:
    values = _coerce(values, data_type)
    col = Column(name=name, data_type=data_type, has_dictionary=has_dictionary)
    if len(values) > 1:
        col.is_sorted = bool(np.all(values[1:] >= values[:-1]))
    if not has_dictionary:
        if data_type == "STRING":
            raise ValueError("raw STRING columns are out of the hot-path scope")
        col.raw_values = np.ascontiguousarray(values)
        return col
    dictionary, ids = np.unique(values, return_inverse=True)
    col.dictionary = dictionary
    col.cardinality = int(len(dictionary))
    col.num_bits = num_bits_per_value(col.cardinality - 1)
    col.fwd_bytes = pack_bits(ids.astype(np.uint32), col.num_bits)
    return col


def create_segment(name, data: Dict[str, np.ndarray], schema: Dict[str, str], no_dictionary_columns=(),
                   multi_value_columns=(), inverted_index_columns=(), range_index_columns=()) -> Segment:
    """Builds an immutable segment from column arrays. schema: column -> data type; a multi-value column's data is a
    sequence of per-doc value arrays. inverted_index_columns / range_index_columns: the table config's index lists
    (SegmentGeneratorConfig.setIndexOn), kept as column metadata for the execution statistics."""
    n = None
    seg = None
    for col_name, dtype in schema.items():
        vals = data[col_name]
        if n is None:
            n = len(vals)
            seg = Segment(name=name, num_docs=n)
        elif len(vals) != n:
            raise ValueError("column %s has %d rows, expected %d" % (col_name, len(vals), n))
        if col_name in multi_value_columns:
            seg.columns[col_name] = build_mv_column(col_name, vals, dtype)
        else:
            seg.columns[col_name] = build_column(col_name, vals, dtype, col_name not in no_dictionary_columns)
    if seg is None:
        seg = Segment(name=name, num_docs=0)
    for c in inverted_index_columns:
        seg.column(c).inverted_index = True
    for c in range_index_columns:
        seg.column(c).range_index = True
    return seg


def segment_from_dict_ids(name, num_docs, specs) -> Segment:
    """Synthetic segment straight from (dictionary, packed bytes): specs = {col: (dtype, dictionary, fwd_bytes)}."""
    seg = Segment(name=name, num_docs=num_docs)
    for col_name, (dtype, dictionary, fwd) in specs.items():
        c = Column(name=col_name, data_type=dtype)
        c.dictionary = dictionary
        c.cardinality = len(dictionary)
        c.num_bits = num_bits_per_value(c.cardinality - 1)
        need = (num_docs * c.num_bits + 7) // 8
        if len(fwd) < need:
            raise ValueError("forward index too short")
        c.fwd_bytes = fwd
        seg.columns[col_name] = c
    return seg
