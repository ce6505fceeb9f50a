"""ctypes binding of include/pinot_amd.h (the C-ABI a Pinot server would bind through FFM/JNI).

There is no CPU fallback: if libpinot_amd.so is missing or a call fails, a PinotAmdError is raised.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpinot_amd.so")

PA_MAX_LEAVES = 16
PA_MAX_OPS = 48
PA_MAX_GROUP_BY = 8
PA_MAX_AGGS = 16

PA_INT, PA_LONG, PA_FLOAT, PA_DOUBLE, PA_STRING, PA_BYTES = range(6)
PA_LEAF_DICT_RANGE, PA_LEAF_DICT_SET, PA_LEAF_RAW_RANGE, PA_LEAF_MV_DICT_RANGE, PA_LEAF_MV_DICT_SET, PA_LEAF_RAW_SET = range(6)
PA_OP_LEAF, PA_OP_AND, PA_OP_OR, PA_OP_NOT = range(4)
PA_AGG_COUNT, PA_AGG_SUM, PA_AGG_MIN, PA_AGG_MAX, PA_AGG_DISTINCTCOUNTHLL, PA_AGG_COUNT_MV, PA_AGG_DISTINCTCOUNT = range(7)
PA_QF_STAGE_ALL = 1
PA_QF_FORCE_GLOBAL = 2
PA_QF_STEPS16 = 1 << 4
PA_QF_STEPS32 = 1 << 5
PA_QF_NO_LAZY = 1 << 6
PA_QF_FORCE_LDS = 1 << 7
PA_QF_RING_SHIFT = 8
PA_QF_WG_SHIFT = 12
PA_QF_DEBUG_STREAM_ONLY = 1 << 16
PA_QF_NO_LANE_MAJOR = 1 << 17
PA_QF_NO_REG_STAGE = 1 << 18
PA_QF_NO_GDENSE_LM = 1 << 15
PA_QF_NO_GD_PACK = 1 << 3
PA_QF_GD_DRAIN_EACH_TILE = 1 << 2
PA_QF_NO_JIT = 1 << 31  # bit 31 of the int32 flags word (engine converts to int32)
PA_QF_NO_BOX_FILTER = 1 << 19
PA_QF_BOX_FILTER = 1 << 20
PA_QF_NO_PARTITION = 1 << 21
PA_QF_PART_SHIFT = 22
PA_QF_NO_SPLIT_EMIT = 1 << 24
PA_QF_NO_LIMIT_WALK = 1 << 25
PA_QF_NO_LANE_ACC = 1 << 26
PA_QF_NO_LANE_HIST = 1 << 27
PA_QF_LAZY_POST = 1 << 28
PA_QF_NO_DENSE_GROUP = 1 << 29
PA_QF_NO_FILTER_STATS = 1 << 30
PA_QF2_NO_COUNT_FREE = 1 << 32  # (engine flags: bits 32.. go to pa_query_spec.flags2)
PA_FOP_EMPTY, PA_FOP_MATCH_ALL, PA_FOP_SORTED, PA_FOP_BITMAP, PA_FOP_SCAN, PA_FOP_AND, PA_FOP_OR, PA_FOP_NOT = range(8)
PA_STATS_NON_SCAN, PA_STATS_HOST = -1, -2
PA_BIT_AND, PA_BIT_OR, PA_BIT_NOT = -1, -2, -3
PA_BIT_PROG_MAX = 64
PA_ACC_COUNT_U64, PA_ACC_SUM_I64, PA_ACC_SUM_F64, PA_ACC_MIN_I64, PA_ACC_MAX_I64, PA_ACC_HLL_U8, \
    PA_ACC_SUM_I64X2, PA_ACC_DOCS_U64, PA_ACC_KEYS_I64, PA_ACC_PRESENCE_U8 = range(10)
ABI_VERSION = 4

# every symbol declared in include/pinot_amd.h
EXPORTED = [
    "pa_abi_version", "pa_device_count", "pa_set_device", "pa_last_error", "pa_host_alloc", "pa_host_free",
    "pa_segment_create", "pa_segment_add_sv_dict_column", "pa_segment_add_mv_dict_column",
    "pa_segment_add_raw_column", "pa_segment_num_docs", "pa_segment_device_bytes", "pa_segment_destroy",
    "pa_query_create", "pa_query_bind_segment", "pa_query_bind_value_remap", "pa_query_prepare", "pa_query_num_keys",
    "pa_query_execute", "pa_query_reset", "pa_query_scan", "pa_query_num_eager_literals", "pa_query_lane_major",
    "pa_query_dense_packed", "pa_query_count_free_emit", "pa_query_partition_keys",
    "pa_query_accumulator_bytes", "pa_query_set_accumulator_buffer", "pa_query_num_sections", "pa_query_section",
    "pa_query_fetch", "pa_query_matched_docs", "pa_query_key_layout", "pa_query_limit_trimming",
    "pa_query_num_groups_limit_reached", "pa_query_stats", "pa_query_leaf_bitmap_words", "pa_query_leaf_bitmaps",
    "pa_bitmap_counts_scratch_bytes", "pa_bitmap_counts", "pa_query_filter_counts",
    "pa_query_plan", "pa_query_column_staged", "pa_query_leap_leaf", "pa_query_leap_counts",
    "pa_query_execution_stats",
    "pa_query_row_bytes", "pa_query_pack_rows", "pa_query_merge_rows", "pa_query_key_words", "pa_query_destroy",
]


class PinotAmdError(RuntimeError):
    pass


class LeafSpec(ctypes.Structure):
    _fields_ = [("column_id", ctypes.c_int32), ("kind", ctypes.c_int32)]


class AggSpec(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("column_id", ctypes.c_int32), ("log2m", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("num_values", ctypes.c_int64)]


PA_AGGF_WIDE_SUM = 1


class QuerySpec(ctypes.Structure):
    _fields_ = [
        ("num_leaves", ctypes.c_int32),
        ("leaves", LeafSpec * PA_MAX_LEAVES),
        ("num_ops", ctypes.c_int32),
        ("ops", ctypes.c_int32 * PA_MAX_OPS),
        ("num_group_by", ctypes.c_int32),
        ("group_by_columns", ctypes.c_int32 * PA_MAX_GROUP_BY),
        ("group_by_cardinality", ctypes.c_int64 * PA_MAX_GROUP_BY),
        ("num_aggs", ctypes.c_int32),
        ("aggs", AggSpec * PA_MAX_AGGS),
        ("flags", ctypes.c_int32),
        ("num_groups_limit", ctypes.c_int32),
        ("hash_keys_bound", ctypes.c_int64),
        ("flags2", ctypes.c_int32),
        ("reserved2", ctypes.c_int32),
    ]


class LeafParams(ctypes.Structure):
    _fields_ = [
        ("lo", ctypes.c_int32), ("hi", ctypes.c_int32), ("negate", ctypes.c_int32), ("reserved", ctypes.c_int32),
        ("lut", ctypes.POINTER(ctypes.c_uint32)),
        ("ilo", ctypes.c_int64), ("ihi", ctypes.c_int64),
        ("dlo", ctypes.c_double), ("dhi", ctypes.c_double),
        ("values", ctypes.c_void_p), ("num_values", ctypes.c_int64),
    ]


_lib = None


def _declare(lib):
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    sig = {
        "pa_abi_version": (ctypes.c_int, []),
        "pa_device_count": (ctypes.c_int, []),
        "pa_set_device": (ctypes.c_int, [ctypes.c_int]),
        "pa_last_error": (ctypes.c_char_p, []),
        "pa_host_alloc": (vp, [u64]),
        "pa_host_free": (None, [vp]),
        "pa_segment_create": (vp, [i32]),
        "pa_segment_add_sv_dict_column": (ctypes.c_int, [vp, i32, vp, u64, i32, i32, i32, vp, vp]),
        "pa_segment_add_mv_dict_column": (ctypes.c_int, [vp, i32, vp, u64, i32, i32, i64, i32, vp, vp]),
        "pa_segment_add_raw_column": (ctypes.c_int, [vp, i32, i32, vp]),
        "pa_segment_num_docs": (i32, [vp]),
        "pa_segment_device_bytes": (u64, [vp]),
        "pa_segment_destroy": (None, [vp]),
        "pa_query_create": (vp, [ctypes.POINTER(QuerySpec), i32]),
        "pa_query_bind_segment": (ctypes.c_int, [vp, i32, vp, ctypes.POINTER(LeafParams), vp]),
        "pa_query_bind_value_remap": (ctypes.c_int, [vp, i32, i32, vp]),
        "pa_query_prepare": (ctypes.c_int, [vp]),
        "pa_query_num_keys": (i64, [vp]),
        "pa_query_execute": (ctypes.c_int, [vp, vp]),
        "pa_query_reset": (ctypes.c_int, [vp, vp]),
        "pa_query_scan": (ctypes.c_int, [vp, vp]),
        "pa_query_num_eager_literals": (i32, [vp]),
        "pa_query_lane_major": (i32, [vp]),
        "pa_query_dense_packed": (i32, [vp]),
        "pa_query_count_free_emit": (i32, [vp]),
        "pa_query_partition_keys": (i32, [vp]),
        "pa_query_accumulator_bytes": (u64, [vp]),
        "pa_query_set_accumulator_buffer": (ctypes.c_int, [vp, vp, u64]),
        "pa_query_num_sections": (i32, [vp]),
        "pa_query_section": (vp, [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i64)]),
        "pa_query_fetch": (i64, [vp, vp, i64, vp, vp, vp]),
        "pa_query_matched_docs": (i64, [vp]),
        "pa_query_key_layout": (ctypes.c_int, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pa_query_limit_trimming": (i32, [vp]),
        "pa_query_num_groups_limit_reached": (ctypes.c_int64, [vp]),
        "pa_query_stats": (ctypes.c_int, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "pa_query_leaf_bitmap_words": (ctypes.c_int64, [vp, i32]),
        "pa_query_leaf_bitmaps": (ctypes.c_int, [vp, i32, vp, vp]),
        "pa_bitmap_counts_scratch_bytes": (i64, [i64]),
        "pa_bitmap_counts": (ctypes.c_int, [vp, i64, i32, i64, vp, i32, vp, i32, vp, vp, vp]),
        "pa_query_filter_counts": (ctypes.c_int, [vp, i32, vp, vp, vp, vp, vp]),
        "pa_query_plan": (ctypes.c_int, [vp] + [ctypes.POINTER(i32)] * 7),
        "pa_query_column_staged": (i32, [vp, i32]),
        "pa_query_leap_leaf": (i32, [vp]),
        "pa_query_leap_counts": (ctypes.c_int, [vp, vp, vp]),
        "pa_query_execution_stats": (ctypes.c_int, [vp, i32, vp, i32, vp, vp, i32, i64, vp, vp, vp]),
        "pa_query_row_bytes": (i64, [vp]),
        "pa_query_key_words": (i32, [vp]),
        "pa_query_pack_rows": (ctypes.c_int, [vp, i32, vp, vp, vp]),
        "pa_query_merge_rows": (ctypes.c_int, [vp, vp, i64, vp, vp, vp]),
        "pa_query_destroy": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def lib():
    """Loads the in-tree HIP extension; raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PinotAmdError("%s is missing: run `python -m pinot_amd.build` (hipcc, gfx950)" % LIB_PATH)
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
        if _lib.pa_abi_version() != ABI_VERSION:
            raise PinotAmdError("ABI version mismatch: %s is stale, rebuild it" % LIB_PATH)
    return _lib


def check(rc, what=""):
    if rc < 0:
        raise PinotAmdError("%s failed (%d): %s" % (what, rc, lib().pa_last_error().decode(errors="replace")))
    return rc


def check_ptr(p, what=""):
    if not p:
        raise PinotAmdError("%s failed: %s" % (what, lib().pa_last_error().decode(errors="replace")))
    return p
