"""Java hashCode restatement behind DISTINCTCOUNTBITMAP (java_hash.py; DistinctCountBitmapAggregationFunction.java:
410-446) on values whose Java hash codes are known, and against the oracle's independent restatement. No GPU."""
import numpy as np
import pytest

import oracle
from pinot_amd import parse_sql
from pinot_amd.java_hash import java_hash_code
from pinot_amd.reduce import final_value
from pinot_amd.segment import create_segment

# (value, type, Java's hashCode)
KNOWN = [("hello", "STRING", 99162322), ("", "STRING", 0), ("Aa", "STRING", 2112), ("BB", "STRING", 2112),
         ("été", "STRING", 227742), (1 << 32, "LONG", 1), (-1, "LONG", 0), (123, "LONG", 123),
         (-5, "INT", -5), (1.0, "DOUBLE", 1072693248), (-0.0, "DOUBLE", -2147483648), (1.0, "FLOAT", 1065353216),
         (float("nan"), "FLOAT", 2143289344), (float("nan"), "DOUBLE", 2146959360)]


@pytest.mark.parametrize("value,dt,want", KNOWN)
def test_known_hash_codes(value, dt, want):
    assert java_hash_code(value, dt) == want
    assert oracle._java_hash(value, dt) == want


def test_distinct_count_bitmap_counts_distinct_hash_codes():
    rng = np.random.default_rng(3)
    n = 4000
    data = {"d": rng.integers(0, 4, n).astype(np.int32),
            "l": (rng.integers(0, 40, n) * (1 << 32) + rng.integers(0, 3, n)).astype(np.int64),
            "s": np.array(["Aa", "BB", "x", "y", "hello"])[rng.integers(0, 5, n)]}
    seg = create_segment("b", data, {"d": "INT", "l": "LONG", "s": "STRING"})
    q = parse_sql("SELECT d, DISTINCTCOUNTBITMAP(l), DISTINCTCOUNT(l), DISTINCTCOUNTBITMAP(s) FROM t GROUP BY d")
    res = oracle.run_query(q, [seg])
    for key, v in res.groups.items():
        vals = set(data["l"][data["d"] == key[0]].tolist())
        assert final_value("DISTINCTCOUNT", v[1]) == len(vals)
        assert final_value("DISTINCTCOUNTBITMAP", v[0]) == len({java_hash_code(x, "LONG") for x in vals}) < len(vals)
        assert final_value("DISTINCTCOUNTBITMAP", v[2]) == 4  # ("Aa" and "BB" share a hash code)
