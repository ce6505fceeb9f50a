"""Pins the CPU oracle to the reference's own golden results (no GPU needed).

Every case in tests/golden/sv_queries.json is a query + expected broker ResultTable copied from the reference's
InterSegment*SingleValueQueriesTest (file:line in the case), run on 2 servers x 2 copies of the reference's test
segment (test_data-sv.avro). The oracle must reproduce every one exactly (AVG within the reference's 1e-5).
"""
import pytest

import oracle
from pinot_amd import parse_sql
from pinot_amd.reduce import final_result_table, merge_intermediate, server_trim
from conftest import golden_rows, rows_match


def _broker(query, segment, servers=2, per_server=2):
    server = server_trim(oracle.run_query(query, [segment] * per_server), query)
    merged = merge_intermediate([server] * servers)
    return final_result_table(merged, query), merged


def test_golden_cases(golden_spec, golden_segment):
    failures = []
    for case in golden_spec["cases"]:
        q = parse_sql(case["sql"])
        got, merged = _broker(q, golden_segment)
        if case["rows"] is not None and not rows_match(golden_rows(got, case), case["rows"], case["delta"]):
            failures.append((case["source"], case["sql"], got[:5], case["rows"][:5]))
        # BrokerResponseNative.isNumGroupsLimitReached: OR over the servers' DataTable metadata
        if "limit_reached" in case and merged.num_groups_limit_reached != case["limit_reached"]:
            failures.append((case["source"], "numGroupsLimitReached", merged.num_groups_limit_reached))
    assert not failures, "\n".join(map(str, failures))


def test_segment_shape(golden_segment):
    # BaseSingleValueQueriesTest.java:55-68 documents these cardinalities (column12 has 9 distinct values in the
    # avro file; the javadoc's 5 is stale)
    card = {c: golden_segment.column(c).cardinality for c in golden_segment.columns}
    assert card["column1"] == 6582 and card["column3"] == 21910 and card["column5"] == 1
    assert card["column6"] == 608 and card["column7"] == 146 and card["column9"] == 1737
    assert card["column11"] == 5 and card["column17"] == 24 and card["column18"] == 1440
    assert card["daysSinceEpoch"] == 2
    assert golden_segment.num_docs == 30000


@pytest.mark.parametrize("nb", [1, 2, 3, 5, 7, 8, 9, 13, 16, 17, 23, 24, 31])
def test_bitset_roundtrip(nb):
    """Segment creator packing == PinotDataBitSet.writeInt restatement; readInt restatement inverts it."""
    import numpy as np
    from pinot_amd.segment import pack_bits
    rng = np.random.default_rng(nb)
    n = 1000 + nb
    vals = rng.integers(0, 1 << nb, size=n, dtype=np.int64).astype(np.int32)
    packed = pack_bits(vals, nb)
    assert packed.tobytes() == oracle.write_ints(vals, nb).tobytes()
    assert np.array_equal(oracle.read_ints(packed, n, nb), vals)


def test_num_bits_per_value():
    """PinotDataBitSet.getNumBitsPerValue javadoc examples (PinotDataBitSet.java:49-56)."""
    from pinot_amd.segment import num_bits_per_value
    assert [num_bits_per_value(v) for v in (0, 1, 2, 9, 113)] == [1, 1, 2, 4, 7]


def test_query_executor_cases(query_executor_spec, query_executor_segments):
    """QueryExecutorTest.java:152-190: the server-level AggregationResultsBlock value over 2 x simpleData200001 + 2
    empty segments (COUNT long, SUM/MIN/MAX double)."""
    for case in query_executor_spec["cases"]:
        res = oracle.run_query(parse_sql(case["sql"]), query_executor_segments)
        assert res.row[0] == case["value"] and type(res.row[0]) is type(case["value"]), (case["source"], res.row)
