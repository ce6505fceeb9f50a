"""Immutable segment model + creator for the columns the hot path reads.

Mirrors the parts of SegmentIndexCreationDriverImpl the scan path depends on:
  * dictionary: sorted unique values (pinot-segment-local/.../creator/impl/SegmentDictionaryCreator.java),
  * dictionary-encoded SV forward index: FixedBitSVForwardIndexWriter bytes, i.e. PinotDataBitSet.writeInt
    layout (pinot-segment-local/.../io/util/PinotDataBitSet.java:143) — value i at stream bits
    [i*nb, (i+1)*nb), MSB-first, nb = PinotDataBitSet.getNumBitsPerValue(cardinality - 1) (:61),
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


def create_segment(name, data: Dict[str, np.ndarray], schema: Dict[str, str], no_dictionary_columns=()) -> Segment:
    """Builds an immutable segment from column arrays. schema: column -> data type."""
    n = None
    seg = None
    for col_name, dtype in schema.items():
        vals = data[col_name]
        if n is None:
            n = len(vals)
            seg = Segment(name=name, num_docs=n)
        elif len(vals) != n:
            raise ValueError("column %s has %d rows, expected %d" % (col_name, len(vals), n))
        seg.columns[col_name] = build_column(col_name, vals, dtype, col_name not in no_dictionary_columns)
    if seg is None:
        seg = Segment(name=name, num_docs=0)
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
