import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def golden_spec():
    with open(os.path.join(GOLDEN, "sv_queries.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_segment(golden_spec):
    """The reference's BaseSingleValueQueriesTest segment, rebuilt by our segment creator."""
    from pinot_amd.segment import create_segment
    data = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    # BaseSingleValueQueriesTest.java:124-125: inverted indexes on column6/7/11/17/18 (column5 and daysSinceEpoch come
    # out sorted): index metadata for the execution statistics only
    return create_segment("testTable_126164076_167572854", {k: data[k] for k in data.files}, golden_spec["schema"],
                          inverted_index_columns=("column6", "column7", "column11", "column17", "column18"))


def golden_rows(got, case):
    """A golden case's result rows as the reference's test compares them: with "extract": "hll_cardinality" each value
    is a serialized HyperLogLog (DISTINCTCOUNTRAWHLL's hex string) whose cardinality is compared
    (InterSegmentAggregationSingleValueQueriesTest.testDistinctCountRawHLL's cardinalityExtractor)."""
    if case.get("extract") != "hll_cardinality":
        return got
    from pinot_amd.hll import HyperLogLog
    return [[HyperLogLog.from_bytes(bytes.fromhex(v)).cardinality() for v in row] for row in got]


def rows_match(got, expected, delta):
    if len(got) != len(expected):
        return False
    for g, e in zip(got, expected):
        if len(g) != len(e):
            return False
        for a, b in zip(g, e):
            if isinstance(b, str) or isinstance(a, str):
                if a != b:
                    return False
            elif delta:
                if abs(float(a) - float(b)) > delta:
                    return False
            elif float(a) != float(b):
                return False
    return True


_TORCH_GPU = []


def pytest_runtest_setup(item):
    """Before the first GPU test: initialise torch's HIP runtime on device 0. Torch's ROCm wheel carries its own HIP
    runtime; when libpinot_amd's (the system ROCm one) initialises the device first, torch later finds no GPU and the
    RCCL (ProcessGroupNCCL) tests cannot start. Order-independent GPU tests need torch first."""
    if item.get_closest_marker("gpu") is not None and not _TORCH_GPU:
        import torch
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda")
        _TORCH_GPU.append(True)


@pytest.fixture(scope="session")
def query_executor_spec():
    with open(os.path.join(GOLDEN, "query_executor.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def query_executor_segments(query_executor_spec):
    """QueryExecutorTest's server: 2 segments of simpleData200001.avro + 2 empty segments (test_empty_data.json)."""
    from pinot_amd.segment import create_segment
    schema = query_executor_spec["schema"]
    data = np.load(os.path.join(GOLDEN, "simple_data.npz"))
    simple = create_segment("testTable_0", {k: data[k] for k in data.files}, schema)
    empty = create_segment("testTable_2", {k: np.zeros(0, np.int32) for k in schema}, schema)
    return [simple if s == "simple" else empty for s in query_executor_spec["segments"]]
