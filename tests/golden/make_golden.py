"""Generates the committed golden fixtures from the reference's OWN test input and expected results.

Run here (needs /root/reference; the GPU box never runs this):  python tests/golden/make_golden.py

  test_data_sv.npz   the 11 columns BaseSingleValueQueriesTest.java:95-104 selects from
                     pinot-core/src/test/resources/data/test_data-sv.avro (30000 rows, no nulls)
  simple_data.npz    dim0/dim1/met of pinot-core/src/test/resources/data/simpleData200001.avro (200001 rows)
  query_executor.json  QueryExecutorTest.java's server-level aggregation results on it
  sv_queries.json    queries + expected broker ResultTables transcribed from
                     pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentAggregationSingleValueQueriesTest.java
                     and InterSegmentGroupBySingleValueQueriesTest.java (source file:line in every case).
                     Those tests run on 2 servers x 2 identical segments (BaseQueriesTest.java:200-230,
                     BaseSingleValueQueriesTest.java:139), i.e. 4 copies of the segment.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import avro_min  # noqa: E402

AVRO = "/root/reference/pinot-core/src/test/resources/data/test_data-sv.avro"
SCHEMA = {  # BaseSingleValueQueriesTest.java:95-104
    "column1": "INT", "column3": "INT", "column5": "STRING", "column6": "INT", "column7": "INT",
    "column9": "INT", "column11": "STRING", "column12": "STRING", "column17": "INT", "column18": "INT",
    "daysSinceEpoch": "INT",
}

AGG = "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentAggregationSingleValueQueriesTest.java"
GBY = "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentGroupBySingleValueQueriesTest.java"
FILTER = (" WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH'"
          " AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076")
GROUP_BY = " GROUP BY column9 ORDER BY v1 DESC, v2 DESC LIMIT 1"

CASES = []


def case(source, sql, rows, delta=0.0, stats=None, limit_reached=None):
    """stats: the testInterSegmentsResult arguments (numDocsScanned, numEntriesScannedInFilter,
    numEntriesScannedPostFilter, numTotalDocs) the reference asserts for this case (QueriesTestUtils.java).
    rows None: the reference asserts no result table; limit_reached: its assert on isNumGroupsLimitReached()."""
    c = {"source": source, "sql": sql, "rows": rows, "delta": delta, "stats": stats}
    if limit_reached is not None:
        c["limit_reached"] = limit_reached
    CASES.append(c)


# the four execution statistics of the aggregation test's shapes (InterSegmentAggregationSingleValueQueriesTest.java):
# no filter / FILTER, aggregation-only / GROUP BY; `post` = numEntriesScannedPostFilter
def st(filtered, post):
    return [24516, 252256, post, 120000] if filtered else [120000, 0, post, 120000]


# ---- InterSegmentAggregationSingleValueQueriesTest
q = "SELECT COUNT(*) FROM testTable"
case(AGG + ":47-54", q, [[120000]], stats=st(0, 0))
case(AGG + ":56-58", q + FILTER, [[24516]], stats=st(1, 0))
gb = " GROUP BY column9 ORDER BY COUNT(*) DESC LIMIT 1"
case(AGG + ":60-63", q + gb, [[64420]], stats=st(0, 120000))
case(AGG + ":65-67", q + FILTER + gb, [[17080]], stats=st(1, 24516))
q = "SELECT MAX(column1) AS v1, MAX(column3) AS v2 FROM testTable"
case(AGG + ":93-102", q, [[2146952047.0, 2147419555.0]], stats=st(0, 0))
case(AGG + ":104-107", q + FILTER, [[2146952047.0, 999813884.0]], stats=st(1, 49032))
case(AGG + ":109-112", q + GROUP_BY, [[2146952047.0, 2146630496.0]], stats=st(0, 360000))
case(AGG + ":114-117", q + FILTER + GROUP_BY, [[2146952047.0, 999813884.0]], stats=st(1, 73548))
q = "SELECT MIN(column1) AS v1, MIN(column3) AS v2 FROM testTable"
gb = " GROUP BY column9 ORDER BY v1, v2 LIMIT 1"
case(AGG + ":122-131", q, [[240528.0, 17891.0]], stats=st(0, 0))
case(AGG + ":133-136", q + FILTER, [[101116473.0, 20396372.0]], stats=st(1, 49032))
case(AGG + ":138-142", q + gb, [[240528.0, 17891.0]], stats=st(0, 360000))
case(AGG + ":144-147", q + FILTER + gb, [[101116473.0, 91804599.0]], stats=st(1, 73548))
q = "SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable"
case(AGG + ":152-159", q, [[129268741751388.0, 129156636756600.0]], stats=st(0, 240000))
case(AGG + ":161-164", q + FILTER, [[27503790384288.0, 12429178874916.0]], stats=st(1, 49032))
case(AGG + ":166-169", q + GROUP_BY, [[69526727335224.0, 69225631719808.0]], stats=st(0, 360000))
case(AGG + ":171-174", q + FILTER + GROUP_BY, [[19058003631876.0, 8606725456500.0]], stats=st(1, 73548))
q = "SELECT AVG(column1) AS v1, AVG(column3) AS v2 FROM testTable"
case(AGG + ":179-186", q, [[1077239514.5949, 1076305306.305]], 1e-5, stats=st(0, 240000))
case(AGG + ":188-192", q + FILTER, [[1121871038.68037, 506982332.96280]], 1e-5, stats=st(1, 49032))
case(AGG + ":194-197", q + GROUP_BY, [[2142595699.0, 334963174.0]], stats=st(0, 360000))
case(AGG + ":199-202", q + FILTER + GROUP_BY, [[2142595699.0, 334963174.0]], stats=st(1, 73548))
q = "SELECT MINMAXRANGE(column1) AS v1, MINMAXRANGE(column3) AS v2 FROM testTable"
case(AGG + ":207-216", q, [[2146711519.0, 2147401664.0]], stats=st(0, 0))
case(AGG + ":218-221", q + FILTER, [[2045835574.0, 979417512.0]], stats=st(1, 49032))
case(AGG + ":223-226", q + GROUP_BY, [[2146711519.0, 2146612605.0]], stats=st(0, 360000))
case(AGG + ":228-231", q + FILTER + GROUP_BY, [[2044094181.0, 979417512.0]], stats=st(1, 73548))
q = "SELECT DISTINCTCOUNT(column1) AS v1, DISTINCTCOUNT(column3) AS v2 FROM testTable"
case(AGG + ":236-245", q, [[6582, 21910]], stats=st(0, 0))
case(AGG + ":247-249", q + FILTER, [[1872, 4556]], stats=st(1, 49032))
case(AGG + ":251-253", q + GROUP_BY, [[3495, 11961]], stats=st(0, 360000))
case(AGG + ":255-257", q + FILTER + GROUP_BY, [[1272, 3289]], stats=st(1, 73548))
q = "SELECT DISTINCTCOUNTHLL(column1) AS v1, DISTINCTCOUNTHLL(column3) AS v2 FROM testTable"
case(AGG + ":262-271", q, [[5977, 23825]], stats=st(0, 0))
case(AGG + ":273-275", q + FILTER, [[1886, 4492]], stats=st(1, 49032))
case(AGG + ":277-279", q + GROUP_BY, [[3592, 11889]], stats=st(0, 360000))
case(AGG + ":281-283", q + FILTER + GROUP_BY, [[1324, 3197]], stats=st(1, 73548))
# testNumGroupsLimit: only numGroupsLimitReached is asserted (no result table, no statistics); the second query runs on
# a server whose InstancePlanMakerImplV2 has numGroupsLimit = 1000 (column1 has 6582 values per segment)
q = "SELECT COUNT(*) FROM testTable GROUP BY column1"
case(AGG + ":765-768", q, None, limit_reached=False)
case(AGG + ":770-774", q + " OPTION(numGroupsLimit=1000)", None, limit_reached=True)
q = "select DISTINCTSUM(column1) as v1, DISTINCTSUM(column3) as v2 from testTable"
case(AGG + ":779-788", q, [[7074556592262.0, 23553878404013.0]], stats=st(0, 0))
case(AGG + ":790-793", q + FILTER, [[2062916453604.0, 2334011146274.0]], stats=st(1, 49032))
case(AGG + ":795-798", q + GROUP_BY, [[3745055692019.0, 12836683389098.0]], stats=st(0, 360000))
case(AGG + ":800-803", q + FILTER + GROUP_BY, [[1397706323624.0, 1686328722268.0]], stats=st(1, 73548))
q = "select DISTINCTAVG(column1) as v1, DISTINCTAVG(column3) as v2 from testTable"
case(AGG + ":808-818", q, [[1074833879.1039197, 1075028681.150753]], stats=st(0, 0))
case(AGG + ":820-824", q + FILTER, [[1101985285.0448718, 512293930.26207197]], stats=st(1, 49032))
case(AGG + ":826-830", q + GROUP_BY, [[2142595699.0, 334963174.0]], stats=st(0, 360000))
case(AGG + ":832-836", q + FILTER + GROUP_BY, [[2142595699.0, 334963174.0]], stats=st(1, 73548))

# ---- InterSegmentGroupBySingleValueQueriesTest.groupByOrderByDataProvider
c11 = [["", 5935285005452.0], ["P", 88832999206836.0], ["gFuH", 63202785888.0], ["o", 18105331533948.0],
       ["t", 16331923219264.0]]
case(GBY + ":66-71", "SELECT column11, SUM(column1) FROM testTable GROUP BY column11 ORDER BY column11", c11, stats=[120000, 0, 240000, 120000])
case(GBY + ":73-77", "SELECT column11, sum(column1) FROM testTable GROUP BY column11 ORDER BY column11 DESC",
     list(reversed(c11)), stats=[120000, 0, 240000, 120000])
case(GBY + ":79-84", "SELECT column11, Sum(column1) FROM testTable GROUP BY column11 ORDER BY column11 LIMIT 3",
     c11[:3], stats=[120000, 0, 240000, 120000])
two = [["", "HEuxNvH", 3789390396216.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
       ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "dJWwFk", 55470665124.0],
       ["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["P", "HEuxNvH", 21998672845052.0],
       ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0], ["P", "MaztCmmxxgguBUxPti", 27177029040008.0],
       ["P", "TTltMtFiRqUjvOG", 4462670055540.0], ["P", "XcBNHe", 120021767504.0]]
case(GBY + ":86-99", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY column11, column12", two, stats=[120000, 0, 360000, 120000])
case(GBY + ":101-110", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY column11, column12 LIMIT 15",
     two + [["P", "dJWwFk", 6224665921376.0], ["P", "fykKFqiw", 1574451324140.0], ["P", "gFuH", 860077643636.0],
            ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0], ["gFuH", "HEuxNvH", 29872400856.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":112-121", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY column11, column12 DESC",
     [["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["", "dJWwFk", 55470665124.0],
      ["", "MaztCmmxxgguBUxPti", 1333941430664.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
      ["", "HEuxNvH", 3789390396216.0], ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0],
      ["P", "gFuH", 860077643636.0], ["P", "fykKFqiw", 1574451324140.0], ["P", "dJWwFk", 6224665921376.0],
      ["P", "XcBNHe", 120021767504.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":123-132", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY column11, sum(column1)",
     [["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["", "dJWwFk", 55470665124.0],
      ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0], ["", "MaztCmmxxgguBUxPti", 1333941430664.0],
      ["", "HEuxNvH", 3789390396216.0], ["P", "XcBNHe", 120021767504.0], ["P", "gFuH", 860077643636.0],
      ["P", "fykKFqiw", 1574451324140.0], ["P", "TTltMtFiRqUjvOG", 4462670055540.0],
      ["P", "dJWwFk", 6224665921376.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":134-157", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY SUM(column1) DESC LIMIT 50",
     [["P", "MaztCmmxxgguBUxPti", 27177029040008.0], ["P", "HEuxNvH", 21998672845052.0],
      ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0], ["P", "oZgnrlDEtjjVpUoFLol", 8345501392852.0],
      ["o", "MaztCmmxxgguBUxPti", 6905624581072.0], ["P", "dJWwFk", 6224665921376.0],
      ["o", "HEuxNvH", 5026384681784.0], ["t", "MaztCmmxxgguBUxPti", 4492405624940.0],
      ["P", "TTltMtFiRqUjvOG", 4462670055540.0], ["t", "HEuxNvH", 4424489490364.0],
      ["o", "KrNxpdycSiwoRohEiTIlLqDHnx", 4051812250524.0], ["", "HEuxNvH", 3789390396216.0],
      ["t", "KrNxpdycSiwoRohEiTIlLqDHnx", 3529048341192.0], ["P", "fykKFqiw", 1574451324140.0],
      ["t", "dJWwFk", 1349058948804.0], ["", "MaztCmmxxgguBUxPti", 1333941430664.0],
      ["o", "dJWwFk", 1152689463360.0], ["t", "oZgnrlDEtjjVpUoFLol", 1039101333316.0],
      ["P", "gFuH", 860077643636.0], ["", "KrNxpdycSiwoRohEiTIlLqDHnx", 733802350944.0],
      ["o", "oZgnrlDEtjjVpUoFLol", 699381633640.0], ["t", "TTltMtFiRqUjvOG", 675238030848.0],
      ["t", "fykKFqiw", 480973878052.0], ["t", "gFuH", 330331507792.0],
      ["o", "TTltMtFiRqUjvOG", 203835153352.0], ["P", "XcBNHe", 120021767504.0],
      ["o", "fykKFqiw", 62975165296.0], ["", "dJWwFk", 55470665124.0],
      ["gFuH", "HEuxNvH", 29872400856.0], ["gFuH", "MaztCmmxxgguBUxPti", 29170832184.0],
      ["", "oZgnrlDEtjjVpUoFLol", 22680162504.0], ["t", "XcBNHe", 11276063956.0],
      ["gFuH", "KrNxpdycSiwoRohEiTIlLqDHnx", 4159552848.0], ["o", "gFuH", 2628604920.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":159-167", "SELECT sum(column1), MIN(column6) FROM testTable GROUP BY column11 ORDER BY column11",
     [[5935285005452.0, 2.96467636E8], [88832999206836.0, 1689277.0], [63202785888.0, 2.96467636E8],
      [18105331533948.0, 2.96467636E8], [16331923219264.0, 1980174.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":169-178", "SELECT column11, column12, SUM(column1) FROM testTable GROUP BY column11, column12 "
     "ORDER BY SUM  (\tcolumn1) DESC LIMIT 3",
     [["P", "MaztCmmxxgguBUxPti", 27177029040008.0], ["P", "HEuxNvH", 21998672845052.0],
      ["P", "KrNxpdycSiwoRohEiTIlLqDHnx", 18069909216728.0]], stats=[120000, 0, 360000, 120000])
c12min = [["XcBNHe", 329467557.0], ["fykKFqiw", 296467636.0], ["gFuH", 296467636.0], ["HEuxNvH", 6043515.0],
          ["MaztCmmxxgguBUxPti", 6043515.0], ["dJWwFk", 6043515.0], ["KrNxpdycSiwoRohEiTIlLqDHnx", 1980174.0],
          ["TTltMtFiRqUjvOG", 1980174.0], ["oZgnrlDEtjjVpUoFLol", 1689277.0]]
case(GBY + ":180-189", "SELECT column12, MIN(column6) FROM testTable GROUP BY column12 "
     "ORDER BY Min(column6) DESC, column12", c12min, stats=[120000, 0, 240000, 120000])
case(GBY + ":191-198", "SELECT column12 FROM testTable GROUP BY column12 ORDER BY Min(column6) DESC, column12",
     [[r[0]] for r in c12min], stats=[120000, 0, 240000, 120000])
case(GBY + ":200-204", "SELECT column12 FROM testTable GROUP BY column12 ORDER BY Min(column6) DESC, "
     "SUM(column1) LIMIT 3", [["XcBNHe"], ["gFuH"], ["fykKFqiw"]], stats=[120000, 0, 360000, 120000])
case(GBY + ":206-213", "SELECT column12, MIN(column6) FROM testTable GROUP BY column12 "
     "ORDER BY Min(column6) DESC, SUM(column1) LIMIT 3",
     [["XcBNHe", 329467557.0], ["gFuH", 296467636.0], ["fykKFqiw", 296467636.0]], stats=[120000, 0, 360000, 120000])
case(GBY + ":215-225", "select column17, count(*) from testTable group by column17 order by column17 limit 15",
     [[83386499, 2924], [217787432, 3892], [227908817, 6564], [402773817, 7304], [423049234, 6556],
      [561673250, 7420], [635942547, 3308], [638936844, 3816], [939479517, 3116], [984091268, 3824],
      [1230252339, 5620], [1284373442, 7428], [1555255521, 2900], [1618904660, 2744], [1670085862, 3388]], stats=[120000, 0, 120000, 120000])

# Object type aggregations (groupByOrderByDataProvider)
g6 = [["", 296467636.0], ["P", 909380310.3521485], ["gFuH", 296467636.0], ["o", 296467636.0], ["t", 526245333.3900426]]
case(GBY + ":244-249", "SELECT column11, AVG(column6) FROM testTable GROUP BY column11  ORDER BY column11", g6,
     stats=[120000, 0, 240000, 120000])
case(GBY + ":251-257", "SELECT column11, AVG(column6) FROM testTable GROUP BY column11 ORDER BY AVG(column6), column11 DESC",
     [["o", 296467636.0], ["gFuH", 296467636.0], ["", 296467636.0], ["t", 526245333.3900426],
      ["P", 909380310.3521485]], stats=[120000, 0, 240000, 120000])
d12 = [["HEuxNvH", 5], ["KrNxpdycSiwoRohEiTIlLqDHnx", 5], ["MaztCmmxxgguBUxPti", 5], ["TTltMtFiRqUjvOG", 3],
       ["XcBNHe", 2], ["dJWwFk", 4], ["fykKFqiw", 3], ["gFuH", 3], ["oZgnrlDEtjjVpUoFLol", 4]]
case(GBY + ":259-267", "SELECT column12, DISTINCTCOUNT(column11) FROM testTable GROUP BY column12 ORDER BY column12", d12,
     stats=[120000, 0, 240000, 120000])
case(GBY + ":269-277", "SELECT column12, DISTINCTCOUNT(column11) FROM testTable GROUP BY column12 "
     "ORDER BY DistinctCount(column11), column12 DESC",
     [["XcBNHe", 2], ["gFuH", 3], ["fykKFqiw", 3], ["TTltMtFiRqUjvOG", 3], ["oZgnrlDEtjjVpUoFLol", 4], ["dJWwFk", 4],
      ["MaztCmmxxgguBUxPti", 5], ["KrNxpdycSiwoRohEiTIlLqDHnx", 5], ["HEuxNvH", 5]], stats=[120000, 0, 240000, 120000])


# ---- QueryExecutorTest (server level: ServerQueryExecutorV1Impl over 2 segments of simpleData200001.avro + 2 empty
# segments from test_empty_data.json; the asserted value is the AggregationResultsBlock's intermediate result)
QE = "pinot-core/src/test/java/org/apache/pinot/core/query/executor/QueryExecutorTest.java"
SIMPLE_AVRO = "/root/reference/pinot-core/src/test/resources/data/simpleData200001.avro"
SIMPLE_SCHEMA = {"dim0": "INT", "dim1": "INT", "met": "INT"}  # SegmentTestUtils.extractSchemaFromAvroWithoutTime
QE_CASES = [
    {"source": QE + ":152-160", "sql": "SELECT COUNT(*) FROM testTable_OFFLINE", "value": 400002},
    {"source": QE + ":162-170", "sql": "SELECT SUM(met) FROM testTable_OFFLINE", "value": 40000200000.0},
    {"source": QE + ":172-180", "sql": "SELECT MAX(met) FROM testTable_OFFLINE", "value": 200000.0},
    {"source": QE + ":182-190", "sql": "SELECT MIN(met) FROM testTable_OFFLINE", "value": 0.0},
]


def main():
    _, srecs = avro_min.read_avro(SIMPLE_AVRO)
    np.savez_compressed(os.path.join(HERE, "simple_data.npz"),
                        **{c: np.array([r[c] for r in srecs], dtype=np.int32) for c in SIMPLE_SCHEMA})
    with open(os.path.join(HERE, "query_executor.json"), "w") as f:
        # the server's segments: 2 x simpleData200001 + 2 empty (QueryExecutorTest.java:76-77)
        json.dump({"schema": SIMPLE_SCHEMA, "segments": ["simple", "simple", "empty", "empty"], "cases": QE_CASES},
                  f, indent=1)
    _, recs = avro_min.read_avro(AVRO)
    cols = {}
    for name, dt in SCHEMA.items():
        vals = [r[name] for r in recs]
        assert all(v is not None for v in vals), name
        cols[name] = np.array(vals, dtype=np.int32) if dt == "INT" else np.array(vals).astype(str)
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **cols)
    with open(os.path.join(HERE, "sv_queries.json"), "w") as f:
        json.dump({"schema": SCHEMA, "copies": 4, "servers": 2, "segments_per_server": 2, "cases": CASES},
                  f, indent=1)
    print("wrote %d rows, %d cases" % (len(recs), len(CASES)))


if __name__ == "__main__":
    main()
