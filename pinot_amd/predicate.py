"""Host-side predicate evaluators: resolve a value-space predicate against ONE segment's dictionary into the
dictId-space leaf the GPU evaluates (the same resolution the reference's PredicateEvaluators perform before
scanning; the GPU then replaces their applySV loops).

  EqPredicate      -> EqualsPredicateEvaluatorFactory.DictionaryBasedEqPredicateEvaluator (dictId == indexOf(v))
  NotEqPredicate   -> NotEqualsPredicateEvaluatorFactory (dictId != indexOf(v))
  InPredicate      -> InPredicateEvaluatorFactory.DictionaryBasedInPredicateEvaluator (matching dictId set)
  NotInPredicate   -> NotInPredicateEvaluatorFactory (complement of the matching set)
  RangePredicate   -> RangePredicateEvaluatorFactory.SortedDictionaryBasedRangePredicateEvaluator:113-150
                      (insertionIndexOf on the sorted dictionary -> [startDictId, endDictId))
Raw (no-dictionary) columns resolve to inclusive value ranges, like the *RawValueBased* evaluators.
"""
import re
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import query as Q
from ._lib import PA_LEAF_DICT_RANGE, PA_LEAF_DICT_SET, PA_LEAF_RAW_RANGE, PA_LEAF_RAW_SET

INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


_JAVA_INTEGER = re.compile(r"[+-]?[0-9]+\Z")


def parse_integral(raw, data_type):
    """Integer.parseInt / Long.parseLong, exactly: an optional sign and decimal digits, within the type's range
    (IntDictionary.insertionIndexOf / RangePredicateEvaluatorFactory.java:80-85 parse the literal this way). Anything
    else — '1.5', '1e3', ' 7', a value past the type's range — is a NumberFormatException in the reference, so the
    query is refused rather than answered for a rounded literal."""
    s = str(raw)
    lo, hi = (INT_MIN, INT_MAX) if data_type == "INT" else (LONG_MIN, LONG_MAX)
    if not _JAVA_INTEGER.match(s) or not lo <= int(s) <= hi:
        raise ValueError("NumberFormatException: %r is not a valid %s literal" % (s, data_type))
    return int(s)


def stored_value(raw, data_type):
    """PredicateUtils.getStoredValue + the type's parse (Integer.parseInt, Long.parseLong, ...)."""
    if data_type in ("INT", "LONG"):
        return parse_integral(raw, data_type)
    if data_type == "FLOAT":
        return np.float32(float(raw))
    if data_type == "DOUBLE":
        return float(raw)
    return str(raw)


@dataclass
class DictLeaf:
    """Per-segment parameters of a dictionary leaf: match = (dictId in [lo, hi) or lut bit) XOR negate."""
    kind: int
    lo: int = 0
    hi: int = 0
    ids: Optional[np.ndarray] = None
    negate: bool = False

    def lut_words(self, cardinality):
        words = np.zeros((cardinality + 31) // 32, dtype=np.uint32)
        if self.ids is not None and len(self.ids):
            ids = np.asarray(self.ids, dtype=np.int64)
            np.bitwise_or.at(words, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
        return words


@dataclass
class RawLeaf:
    ilo: int = LONG_MIN
    ihi: int = LONG_MAX
    dlo: float = -np.inf
    dhi: float = np.inf
    negate: bool = False
    kind: int = PA_LEAF_RAW_RANGE
    values: object = None  # RAW_SET: int64 (INT/LONG) or float64 (FLOAT/DOUBLE) sorted unique values


def _ids_leaf(ids, negate):
    ids = np.unique(np.asarray(ids, dtype=np.int64))
    if len(ids) == 0:
        return DictLeaf(PA_LEAF_DICT_RANGE, 0, 0, None, negate)
    if ids[-1] - ids[0] + 1 == len(ids):
        return DictLeaf(PA_LEAF_DICT_RANGE, int(ids[0]), int(ids[-1]) + 1, None, negate)
    return DictLeaf(PA_LEAF_DICT_SET, 0, 0, ids.astype(np.int32), negate)


def dictionary_leaf(pred, column) -> DictLeaf:
    dt = column.data_type
    if isinstance(pred, Q.EqPredicate):
        i = column.index_of(stored_value(pred.value, dt))
        return DictLeaf(PA_LEAF_DICT_RANGE, i, i + 1) if i >= 0 else DictLeaf(PA_LEAF_DICT_RANGE, 0, 0)
    if isinstance(pred, Q.NotEqPredicate):
        i = column.index_of(stored_value(pred.value, dt))
        if i < 0:
            return DictLeaf(PA_LEAF_DICT_RANGE, 0, column.cardinality)
        return DictLeaf(PA_LEAF_DICT_RANGE, i, i + 1, None, True)
    if isinstance(pred, (Q.InPredicate, Q.NotInPredicate)):
        ids = [column.index_of(stored_value(v, dt)) for v in pred.values]
        ids = [i for i in ids if i >= 0]
        return _ids_leaf(ids, isinstance(pred, Q.NotInPredicate))
    if isinstance(pred, Q.RangePredicate):
        # SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:113-150)
        if pred.lower == Q.UNBOUNDED:
            start = 0
        else:
            ins = column.insertion_index_of(stored_value(pred.lower, dt))
            if ins < 0:
                start = -(ins + 1)
            else:
                start = ins if pred.lower_inclusive else ins + 1
        if pred.upper == Q.UNBOUNDED:
            end = column.cardinality
        else:
            ins = column.insertion_index_of(stored_value(pred.upper, dt))
            if ins < 0:
                end = -(ins + 1)
            else:
                end = ins + 1 if pred.upper_inclusive else ins
        if end < start:
            end = start
        return DictLeaf(PA_LEAF_DICT_RANGE, start, end)
    if isinstance(pred, Q.RegexpLikePredicate):
        # DictionaryBasedRegexpLikePredicateEvaluator (RegexpLikePredicateEvaluatorFactory.java): STRING / JSON
        # dictionaries only, applySV(dictId) = the pattern found in the value (Matcher.find(); Python's re.search on
        # the patterns both regex dialects read alike). Resolved once per segment to the matching dictIds
        if dt not in ("STRING", "JSON"):
            raise ValueError("REGEXP_LIKE: unsupported data type %s" % dt)
        rx = re.compile(pred.pattern)
        return _ids_leaf([i for i, v in enumerate(column.dictionary) if rx.search(str(v))], False)
    raise TypeError("unsupported predicate %r" % (pred,))


def raw_leaf(pred, column) -> RawLeaf:
    """Inclusive bounds for a raw-value range/eq predicate (Int/Long/Float/DoubleRawValueBased evaluators); an IN /
    NOT IN list is one RAW_SET leaf of its stored values, sorted and unique (RawValueBasedInPredicateEvaluatorFactory.java:
    the values parsed with the column type's parse into a set; FLOAT values as the stored float, widened)."""
    dt = column.data_type
    integral = dt in ("INT", "LONG")
    lo_min, hi_max = (INT_MIN, INT_MAX) if dt == "INT" else (LONG_MIN, LONG_MAX)
    if isinstance(pred, (Q.InPredicate, Q.NotInPredicate)):
        vals = [stored_value(v, dt) for v in pred.values]
        arr = (np.unique(np.asarray(vals, dtype=np.int64)) if integral else
               np.unique(np.asarray([float(v) for v in vals], dtype=np.float64)))
        if not integral:
            arr = arr[~np.isnan(arr)]
        return RawLeaf(negate=isinstance(pred, Q.NotInPredicate), kind=PA_LEAF_RAW_SET, values=arr)
    if isinstance(pred, (Q.EqPredicate, Q.NotEqPredicate)):
        v = stored_value(pred.value, dt)
        neg = isinstance(pred, Q.NotEqPredicate)
        return RawLeaf(v, v, negate=neg) if integral else RawLeaf(dlo=float(v), dhi=float(v), negate=neg)
    if isinstance(pred, Q.RangePredicate):
        if integral:
            lo = lo_min if pred.lower == Q.UNBOUNDED else stored_value(pred.lower, dt) + (0 if pred.lower_inclusive else 1)
            hi = hi_max if pred.upper == Q.UNBOUNDED else stored_value(pred.upper, dt) - (0 if pred.upper_inclusive else 1)
            return RawLeaf(ilo=lo, ihi=hi)
        ftype = np.float32 if dt == "FLOAT" else np.float64
        if pred.lower == Q.UNBOUNDED:
            lo = -np.inf
        else:
            lo = ftype(stored_value(pred.lower, dt))
            if not pred.lower_inclusive:
                lo = np.nextafter(lo, ftype(np.inf))
        if pred.upper == Q.UNBOUNDED:
            hi = np.inf
        else:
            hi = ftype(stored_value(pred.upper, dt))
            if not pred.upper_inclusive:
                hi = np.nextafter(hi, ftype(-np.inf))
        return RawLeaf(dlo=float(lo), dhi=float(hi))
    raise TypeError("unsupported raw predicate %r" % (pred,))


