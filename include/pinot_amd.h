/*
 * pinot_amd.h — C-ABI of the MI355X-native segment query hot path.
 *
 * This is the drop-in boundary a Pinot server binds (Java FFM / JNI).
 * Everything above it (QueryContext, PredicateEvaluator, Dictionary, DataTable building,
 * broker reduce) stays in the host language; everything below it runs as hand-written HIP
 * on gfx950. Plain pointers and sizes only — no torch, no C++ types.
 *
 * Reference interfaces replaced (all paths relative to /root/reference):
 *
 *  pa_segment_add_sv_dict_column
 *      replaces the device-side role of
 *      pinot-segment-local/.../readers/forward/FixedBitSVForwardIndexReaderV2.java:38 (ctor over the
 *      PinotDataBuffer) and io/reader/impl/FixedBitIntReader.java:51 (getReader): the caller passes the
 *      forward-index bytes exactly as written by FixedBitSVForwardIndexWriter (big-endian, MSB-first,
 *      io/util/PinotDataBitSet.java:80 layout) and the dictionary values
 *      (segment-spi/.../index/reader/Dictionary.java getLongValue/getDoubleValue).
 *  pa_segment_add_mv_dict_column
 *      replaces readers/forward/FixedBitMVForwardIndexReader.java:56 (chunk offsets + row-start bitmap
 *      + bit-packed values, same bytes).
 *  pa_segment_add_raw_column
 *      replaces the raw (no-dictionary) fixed-width forward index readers
 *      (readers/forward/FixedByteChunkSVForwardIndexReader.java) — values are passed decoded.
 *  pa_query_* (spec, bind, execute, fetch)
 *      replaces, for one segment set on one GPU, the per-segment operator chain
 *        pinot-core/.../operator/filter/ScanBasedFilterOperator.java + dociditerators/SVScanDocIdIterator.java:76
 *        operator/filter/BitmapBasedFilterOperator.java, AndFilterOperator.java, OrFilterOperator.java,
 *        NotFilterOperator.java (the filter tree, evaluated in dictId space from
 *        operator/filter/predicate/{Range,In,Equals,NotIn,NotEquals}PredicateEvaluatorFactory.java ranges / matching-dictId sets),
 *        operator/query/AggregationOperator.java and operator/query/GroupByOperator.java:84
 *        (query/aggregation/groupby/DefaultGroupByExecutor.java:140 process(),
 *         DictionaryBasedGroupKeyGenerator.java:233 raw-key generation,
 *         aggregation/function/{Count,Sum,Min,Max,DistinctCountHLL}AggregationFunction.java
 *         aggregateGroupBySV / aggregate),
 *      and the in-server merge of those partial results
 *        operator/combine/AggregationCombineOperator.java, GroupByCombineOperator.java:110
 *      (segments of one GPU accumulate into ONE table-wide key space, so no per-segment merge is needed).
 *  pa_query_accumulators / layout
 *      exposes the device accumulators so the cross-GPU merge of partial aggregates runs as an RCCL
 *      reduce (SUM for COUNT/SUM, MIN, MAX, MAX for HLL registers) — the multi-GPU analogue of
 *      GroupByCombineOperator's IndexedTable upsert/merge.
 *
 * Error convention: functions returning int return 0 on success and a negative PA_E* code on error;
 * pa_last_error() returns a thread-local message. Functions returning pointers return NULL on error.
 */
#ifndef PINOT_AMD_H_
#define PINOT_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PA_ABI_VERSION 4

/* limits of one query shape */
#define PA_MAX_LEAVES 16
#define PA_MAX_OPS 48
#define PA_MAX_GROUP_BY 8
#define PA_MAX_AGGS 16

/* error codes */
#define PA_OK 0
#define PA_EINVAL (-1)
#define PA_EHIP (-2)
#define PA_ENOMEM (-3)
#define PA_EUNSUPPORTED (-4)

/* stored value types: org.apache.pinot.spi.data.FieldSpec.DataType#getStoredType */
#define PA_INT 0
#define PA_LONG 1
#define PA_FLOAT 2
#define PA_DOUBLE 3
#define PA_STRING 4
#define PA_BYTES 5

/* filter leaf kinds (how a predicate is evaluated on the GPU; resolution into dictId space happens in
 * the host's PredicateEvaluator exactly as in the reference) */
#define PA_LEAF_DICT_RANGE 0 /* lo <= dictId < hi   (SortedDictionaryBasedRangePredicateEvaluator, EQ)   */
#define PA_LEAF_DICT_SET 1   /* bit dictId of lut set (IN / NOT IN / unsorted range matching-dictId set)  */
#define PA_LEAF_RAW_RANGE 2  /* ilo<=v<=ihi (INT/LONG) or dlo<=v<=dhi (FLOAT/DOUBLE) on a raw column       */
#define PA_LEAF_MV_DICT_RANGE 3 /* MV column: any value with lo <= dictId < hi (MVScanDocIdIterator)      */
#define PA_LEAF_MV_DICT_SET 4   /* MV column: any value whose bit is set in lut                            */
#define PA_LEAF_RAW_SET 5       /* raw column: v is one of the leaf's num_values values (IN / NOT IN on a no-dictionary
                                   column: RawValueBasedInPredicateEvaluatorFactory.java's value sets), any list size */

/* postfix filter program opcodes; PA_OP_LEAF carries the leaf index in bits 8..15 */
#define PA_OP_LEAF 0
#define PA_OP_AND 1
#define PA_OP_OR 2
#define PA_OP_NOT 3

/* aggregation types (AggregationFunctionType) */
#define PA_AGG_COUNT 0
#define PA_AGG_SUM 1
#define PA_AGG_MIN 2
#define PA_AGG_MAX 3
#define PA_AGG_DISTINCTCOUNTHLL 4
#define PA_AGG_COUNT_MV 5 /* COUNTMV: number of values of an MV column (AVGMV = SUM over an MV column / COUNTMV) */
#define PA_AGG_DISTINCTCOUNT 6 /* exact DISTINCTCOUNT over a dictionary-encoded column: per group, one presence byte per
                                  table-wide value id of the column (pa_agg_spec.num_values of them; segment dictIds are
                                  mapped by pa_query_bind_value_remap) — the value set of DistinctCountAggregationFunction
                                  (BaseDistinctAggregateAggregationFunction) as a bitmap over the table's values */
/* SUM / MIN / MAX / DISTINCTCOUNTHLL over a multi-value column aggregate every value of the doc (SUMMV, MINMV, MAXMV,
 * DISTINCTCOUNTHLLMV); a multi-value group-by column expands a doc into one key per value (cartesian product over
 * several MV columns), as DictionaryBasedGroupKeyGenerator.getIntRawKeys does. */

/* ---------------------------------------------------------------- device / errors */
int pa_abi_version(void);
int pa_device_count(void);
int pa_set_device(int device);
const char* pa_last_error(void);
/* Page-locked host memory of the library's runtime, for fetch output arrays: pa_query_fetch then copies each result
 * column straight into it by DMA (a pooled buffer the caller reuses across fetches). NULL on failure. */
void* pa_host_alloc(uint64_t bytes);
void pa_host_free(void* p);

/* ---------------------------------------------------------------- segments (HBM resident) */
typedef struct pa_segment pa_segment;

pa_segment* pa_segment_create(int32_t num_docs);

/* fwd_index: FixedBitSVForwardIndexWriter bytes, length must equal ceil(num_docs*num_bits/8)
 * (FixedBitIntReaderWriter.java:31 precondition). dict_values: int64[cardinality] for INT/LONG,
 * double[cardinality] for FLOAT/DOUBLE, NULL for STRING/BYTES. dict_hashes (nullable): MurmurHash
 * (stream-lib 2.9.8 MurmurHash.hash(Object)) of every dictionary value, required only to run
 * DISTINCTCOUNTHLL on STRING/BYTES dictionaries (numeric ones are hashed on the GPU). */
int pa_segment_add_sv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value,
                                  int32_t cardinality, int32_t value_type, const void* dict_values,
                                  const int32_t* dict_hashes);

/* fwd_index: FixedBitMVForwardIndexReader layout (chunk offsets | row-start bitmap | bit-packed values). */
int pa_segment_add_mv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value,
                                  int32_t cardinality, int64_t total_num_values, int32_t value_type,
                                  const void* dict_values, const int32_t* dict_hashes);

/* values: int32[num_docs] (INT), int64 (LONG), float (FLOAT), double (DOUBLE). */
int pa_segment_add_raw_column(pa_segment* seg, int32_t column_id, int32_t value_type,
                              const void* values);

int32_t pa_segment_num_docs(const pa_segment* seg);
uint64_t pa_segment_device_bytes(const pa_segment* seg);
void pa_segment_destroy(pa_segment* seg);

/* ---------------------------------------------------------------- query shape */
typedef struct {
  int32_t column_id;
  int32_t kind; /* PA_LEAF_* */
} pa_leaf_spec;

typedef struct {
  int32_t type;      /* PA_AGG_* */
  int32_t column_id; /* ignored for COUNT */
  int32_t log2m;     /* DISTINCTCOUNTHLL only (CommonConstants.Helix.DEFAULT_HYPERLOGLOG_LOG2M = 8) */
  int32_t flags;     /* PA_AGGF_* */
  int64_t num_values; /* DISTINCTCOUNT: size of the column's table-wide value dictionary (ignored otherwise) */
} pa_agg_spec;

/* SUM over an INT/LONG column: keep the exact 96-bit (low 32 unsigned, high 32 signed) pair accumulator
 * (PA_ACC_SUM_I64X2) even when every value of the bound segments fits int32. A multi-GPU query sets it on every rank
 * when any rank holds a value outside int32, so all ranks get the same accumulator layout for the RCCL reduce. */
#define PA_AGGF_WIDE_SUM 1

typedef struct {
  int32_t num_leaves;
  pa_leaf_spec leaves[PA_MAX_LEAVES];
  int32_t num_ops; /* 0 = match all (MatchAllFilterOperator) */
  int32_t ops[PA_MAX_OPS];
  int32_t num_group_by; /* 0 = aggregation-only query */
  int32_t group_by_columns[PA_MAX_GROUP_BY];
  int64_t group_by_cardinality[PA_MAX_GROUP_BY]; /* size of the table-wide key space per column; 0 for a raw
                                                     (no-dictionary) column, grouped by value
                                                     (NoDictionarySingle/MultiColumnGroupKeyGenerator) */
  int32_t num_aggs;
  pa_agg_spec aggs[PA_MAX_AGGS];
  int32_t flags; /* PA_QF_* */
  int32_t num_groups_limit; /* numGroupsLimit (QueryOptionsUtils / InstancePlanMakerImplV2, default 100000); 0 = none.
                               When some segment can hold that many distinct groups, the reference's first-seen trimming
                               runs on the GPU (DictionaryBasedGroupKeyGenerator IntGroupIdMap.getGroupId :992-1017) */
  int64_t hash_keys_bound; /* hashed key spaces: the table holds at least 2 x this many keys (0 = size from the bound
                              segments alone). A multi-GPU query passes the largest per-rank bound of all ranks so every
                              rank's table can hold its share of the cross-GPU merge (parallel.table_layout) */
  int32_t flags2; /* PA_QF2_* */
  int32_t reserved2;
} pa_query_spec;

#define PA_QF_STAGE_ALL 1  /* stage post-filter columns through LDS even when a filter exists */
#define PA_QF_FORCE_GLOBAL 2 /* force global-memory accumulators (testing the fallback) */
/* tuning overrides of the tile planner (0 = automatic) */
#define PA_QF_STEPS16 (1 << 4)        /* 1024-doc wave tiles */
#define PA_QF_STEPS32 (1 << 5)        /* 2048-doc wave tiles */
#define PA_QF_NO_LAZY (1 << 6)        /* evaluate every filter clause on staged tiles (no late materialisation) */
#define PA_QF_FORCE_LDS (1 << 7)      /* LDS-privatised accumulators even for sparse results (when they fit) */
#define PA_QF_RING_SHIFT 8            /* bits 8..11: tile images per wave (2..8) */
#define PA_QF_WG_SHIFT 12             /* bits 12..14: workgroups per CU (1..4) */
#define PA_QF_NO_GDENSE_LM (1 << 15)      /* dense GROUP BY kernel: the step-major walk (ds_read2 per doc and column) instead
                                             of the lane-major one (each lane unpacks its 16 docs of every column) */
#define PA_QF_NO_JIT (1u << 31)          /* never the query-shape specialised dense kernel (gdl_jit.hip); also PA_NO_JIT=1 */
#define PA_QF_GD_DRAIN_EACH_TILE (1 << 2) /* testing: packed dense accumulation drains each wave's rows after every tile */
#define PA_QF_NO_GD_PACK (1 << 3)         /* dense GROUP BY, lane-major walk: one LDS atomic per aggregation and matching doc
                                             instead of one packed word (COUNT + SUM terms) per matching doc */
#define PA_QF_DEBUG_STREAM_ONLY (1 << 16) /* measurement only: stream the tiles, skip decode (results invalid) */
#define PA_QF_NO_LANE_MAJOR (1 << 17)     /* use the step-major scan kernel even when the lane-major one applies */
#define PA_QF_NO_REG_STAGE (1 << 18)      /* dense GROUP BY kernel: tiles staged by the LDS-DMA ring only, never through
                                             VGPRs (the register-staged variants keep more bytes in flight beside large
                                             LDS tables) */
#define PA_QF_NO_BOX_FILTER (1 << 19)     /* dense GROUP BY kernel: evaluate the filter even when it is exactly the group-key
                                             box (unit range clauses on group-by columns), then walk the matching docs */
#define PA_QF_BOX_FILTER (1 << 20)        /* dense GROUP BY kernel: take the key box as the filter (every doc box-checked
                                             instead of filter + walk) when it is exactly the filter; opt-in */
#define PA_QF_NO_PARTITION (1 << 21)      /* high-cardinality dense GROUP BY: per-doc global atomics, not partitioned */
#define PA_QF_NO_SPLIT_EMIT (1 << 24)     /* partitioned aggregation with both record streams: one emit kernel for both
                                             (default: a V launch and an H launch, each holding only its own bins) */
#define PA_QF_NO_LIMIT_WALK (1 << 25)     /* numGroupsLimit: first-position + sort trimming even where the prefix walk applies */
#define PA_QF_NO_LANE_ACC (1 << 26)       /* aggregation-only query: LDS/global accumulators instead of per-lane registers */
#define PA_QF_NO_LANE_HIST (1 << 27)      /* aggregation-only SUM over a shared dictionary: gather each doc's value instead
                                             of counting dictIds in an LDS histogram */
#define PA_QF_LAZY_POST (1 << 28)         /* post-filter columns (group-by keys, aggregated values) read per matching doc
                                             from HBM at any filter density, never staged with the filter columns */
#define PA_QF_NO_DENSE_GROUP (1 << 29)    /* filter + GROUP BY over a small key space: the LDS strategy (post-filter
                                             columns per matching doc from HBM) instead of the dense group-by kernel
                                             (every column staged, value dictionaries and remaps in LDS) */
#define PA_QF_NO_FILTER_STATS (1 << 30)   /* the scan does NOT count what the execution statistics of an AND of two scan
                                             leaves need (by default it does wherever that fused count applies:
                                             pa_query_leap_leaf / pa_query_leap_counts / pa_query_execution_stats) */
#define PA_QF2_NO_COUNT_FREE 1         /* partitioned plans: the count + emit passes even where the count-free emit
                                           (pve_jit.hip, pa_query_count_free_emit) applies */
#define PA_QF_PART_SHIFT 22              /* bits 22..23: LDS per partition of the partitioned aggregation (0 = auto,
                                             1 = 64 KiB, 2 = 96 KiB, 3 = 144 KiB): larger partitions = fewer record
                                             write fronts per XCD */

/* per-(segment, leaf) parameters in that segment's dictId space */
typedef struct {
  int32_t lo, hi;       /* DICT_RANGE: lo <= dictId < hi */
  int32_t negate;       /* result XOR negate */
  int32_t reserved;
  const uint32_t* lut;  /* DICT_SET: host bitmap, ceil(cardinality/32) words, bit (id&31) of word id>>5 */
  int64_t ilo, ihi;     /* RAW_RANGE on INT/LONG, inclusive */
  double dlo, dhi;      /* RAW_RANGE on FLOAT/DOUBLE, inclusive */
  const void* values;   /* RAW_SET: host int64_t[num_values] (INT/LONG column) or double[num_values] (FLOAT/DOUBLE:
                           the stored float widened), strictly ascending; copied at bind */
  int64_t num_values;
} pa_leaf_params;

typedef struct pa_query pa_query;

pa_query* pa_query_create(const pa_query_spec* spec, int32_t num_segments);

/* group_remaps[j]: host int32[segment cardinality of group_by_columns[j]] mapping the segment's dictId
 * to the table-wide key id of that column (NULL = identity). */
int pa_query_bind_segment(pa_query* q, int32_t index, const pa_segment* seg,
                          const pa_leaf_params* leaf_params, const int32_t* const* group_remaps);

/* DISTINCTCOUNT aggregation `agg` on the segment bound at `index`: remap[d] = the table-wide value id of the segment's
 * dictId d (int32[segment cardinality]; NULL = identity, the segment's dictionary IS the table-wide one). Call after
 * pa_query_bind_segment, before pa_query_prepare. */
int pa_query_bind_value_remap(pa_query* q, int32_t index, int32_t agg, const int32_t* remap);

/* Uploads per-segment parameters, builds the tile schedule and HLL lookup tables, sizes the
 * accumulators. Must be called once after every segment is bound. */
int pa_query_prepare(pa_query* q);

/* Number of keys of the table-wide key space (1 for aggregation-only queries). */
int64_t pa_query_num_keys(const pa_query* q);

/* Zeroes the accumulators and runs the fused scan (filter + group-key + aggregate) over every bound
 * segment on `stream` (hipStream_t, NULL = default stream). Asynchronous. Equivalent to pa_query_reset followed by
 * pa_query_scan (the two halves exist so a caller can time the scan kernel alone). */
int pa_query_execute(pa_query* q, void* stream);
int pa_query_reset(pa_query* q, void* stream);
int pa_query_scan(pa_query* q, void* stream);

/* Accumulator sections, for the cross-GPU RCCL reduce. section kinds: */
#define PA_ACC_COUNT_U64 0 /* reduce SUM */
#define PA_ACC_SUM_I64 1   /* reduce SUM */
#define PA_ACC_SUM_F64 2   /* reduce SUM */
#define PA_ACC_MIN_I64 3   /* reduce MIN (ordered encoding for floating values) */
#define PA_ACC_MAX_I64 4   /* reduce MAX */
#define PA_ACC_HLL_U8 5    /* reduce MAX; one byte per register: [key << log2m | register] */
#define PA_ACC_SUM_I64X2 6 /* reduce SUM; [2k] = sum of low 32 bits (unsigned), [2k+1] = sum of high 32 bits */
#define PA_ACC_DOCS_U64 7  /* reduce SUM; [0] docs that passed the filter (numDocsScanned), [1] group-table overflows,
                              [2] segments whose distinct groups reached numGroupsLimit, [3] internal consistency
                              errors (must stay 0; fetch fails otherwise) */
#define PA_ACC_KEYS_I64 8  /* hashed key space only: slot -> packed key (INT64_MAX = empty); not element-wise
                              reducible across GPUs (slots differ): merge fetched groups by key instead */
#define PA_ACC_PRESENCE_U8 9 /* reduce MAX; DISTINCTCOUNT: [key * stride + value id] = 1 if the group saw the value,
                                stride = num_values rounded up to 16 bytes */
/* All sections live in one device block of pa_query_accumulator_bytes() bytes (256-byte aligned sections).
 * pa_query_set_accumulator_buffer lets the caller own that block (e.g. memory its collective library
 * registered) instead of the library: call after pa_query_prepare; `bytes` must be >= the size. */
uint64_t pa_query_accumulator_bytes(const pa_query* q);
int pa_query_set_accumulator_buffer(pa_query* q, void* device_buffer, uint64_t bytes);
int32_t pa_query_num_sections(const pa_query* q);
/* returns device pointer, writes kind and element count */
void* pa_query_section(const pa_query* q, int32_t section, int32_t* kind, int64_t* num_elements);

/* Compacts the non-empty keys (count > 0) in ascending key order and copies them to the host.
 * out_keys: int64[capacity]; out_counts: int64[capacity]; out_aggs[i]: double[capacity] for
 * COUNT/SUM/MIN/MAX (the reference's intermediate type), uint8[capacity << log2m] for HLL registers.
 * For aggregation-only queries key 0 is always returned (count may be 0).
 * Returns the number of groups (may exceed capacity: then only `capacity` were written), <0 on error.
 * capacity = 0 (output pointers may be NULL) only counts the groups — for large key spaces just the GPU count pass —
 * so a caller can size its arrays exactly before the real fetch. Synchronises `stream`. */
int64_t pa_query_fetch(pa_query* q, void* stream, int64_t capacity, int64_t* out_keys,
                       int64_t* out_counts, void* const* out_aggs);

/* numDocsScanned captured by the last pa_query_fetch (docs that passed the filter; with a multi-value group-by this
 * differs from the sum of the group counts), <0 on error. */
int64_t pa_query_matched_docs(const pa_query* q);

/* numGroupsLimit: 0 if no segment can reach the limit; 1 if the first-position + sort trimming passes run; 2 if the
 * prefix walk runs (SV group-by over a direct key space: limit_walk_kernel + admission inside the scan); <0 if not
 * prepared. */
int32_t pa_query_limit_trimming(const pa_query* q);
/* Segments whose distinct groups reached numGroupsLimit in the last pa_query_fetch (the reference's
 * numGroupsLimitReached is this > 0: GroupByOperator.java:112 per segment, GroupByCombineOperator.java:154 OR), <0 on
 * error. */
int64_t pa_query_num_groups_limit_reached(const pa_query* q);

/* Per-leaf doc bitmaps of one bound segment, for the execution statistics (numEntriesScannedInFilter): the reference
 * counts the docs its filter operators scan (SVScanDocIdIterator.java:76-142: next / advance / applyAnd; AndDocIdSet /
 * OrDocIdSet iterator construction), which depends on which docs each predicate matches and on the segment's indexes,
 * so the host restates that accounting (pinot_amd/filter_stats.py) over these bitmaps. Writes, for every filter leaf l
 * of the spec (pa_query_spec.leaves order), pa_query_leaf_bitmap_words(q, segment) 32-bit words at device_out +
 * l * words: bit (doc & 31) of word (doc >> 5) = the leaf's predicate (with its per-segment negate) on doc.
 * Asynchronous on `stream`. */
int64_t pa_query_leaf_bitmap_words(const pa_query* q, int32_t segment);
int pa_query_leaf_bitmaps(pa_query* q, int32_t segment, uint32_t* device_out, void* stream);

/* Counts over leaf doc bitmaps (pa_query_leaf_bitmaps' layout: leaf l's `words` words at device_bitmaps + l * words,
 * `words` a multiple of 4 covering num_docs)
 * for the execution statistics' closed forms (pinot_amd/filter_stats.py device path), replacing the doc-by-doc replay of
 * the reference's iterators (SVScanDocIdIterator.java:76-142, AndDocIdIterator.java:39-73, AndDocIdSet.java:72-186).
 * prog_a / prog_b: postfix programs over the leaves (a token >= 0 pushes leaf `token`; PA_BIT_AND / PA_BIT_OR pop two
 * masks and push their AND / OR; PA_BIT_NOT complements the top within num_docs; at most PA_BIT_PROG_MAX tokens, stack
 * depth 16, exactly one mask left). ADDS into device_out[0..3] (int64, caller-zeroed): popcount(A), popcount(B),
 * popcount(A & B), and — when len_b > 0 — the leaps of AND(A, B)'s leap-frogging over two scan iterators (labelled
 * docs A-only / B-only / both, in doc order: an A-only doc after a both-doc or at the segment start, or an A-only /
 * B-only doc after the other, starts a leap), from which numEntriesScannedInFilter = num_docs + popcount(A & B) + leaps.
 * device_scratch: pa_bitmap_counts_scratch_bytes(words) bytes. Returns when the counts are written (synchronises
 * `stream`). */
#define PA_BIT_AND (-1)
#define PA_BIT_OR (-2)
#define PA_BIT_NOT (-3)
#define PA_BIT_PROG_MAX 64
int64_t pa_bitmap_counts_scratch_bytes(int64_t words);
int pa_bitmap_counts(const uint32_t* device_bitmaps, int64_t words, int32_t num_leaves, int64_t num_docs,
                     const int32_t* prog_a, int32_t len_a, const int32_t* prog_b, int32_t len_b, void* device_scratch,
                     int64_t* device_out, void* stream);
/* The same counts for many (segment, program A, program B) requests of a prepared query in one pass: the leaf
 * bitmaps of every requested segment (pa_query_leaf_bitmaps) in one launch, then the count kernels for all requests
 * in one launch each. Request r: segments[r], its programs at programs + r * 2 * PA_BIT_PROG_MAX (A, then B at
 * + PA_BIT_PROG_MAX), lengths[2r], lengths[2r + 1] (B may be empty). Writes out[4r .. 4r + 3] (host memory) and
 * returns when they are written (synchronises `stream`). Device scratch is owned by the query. */
int pa_query_filter_counts(pa_query* q, int32_t num_requests, const int32_t* segments, const int32_t* programs,
                           const int32_t* lengths, int64_t* out, void* stream);
/* Execution statistics fused into the scan (PA_QF_FILTER_STATS). When the filter is an AND of two single-value scan
 * leaves, one evaluated on whole tiles (E, sparse) and one per E doc (Z), the scan also counts per segment the docs
 * that matched and the leaps of AndDocIdIterator(A = Z, B = E) (the counts pa_query_filter_counts gives for programs
 * A = [Z], B = [E]): pa_query_leap_leaf returns E's leaf index (spec order) when the scan counts them, else -1.
 * pa_query_leap_counts writes out[3 s .. 3 s + 2] = (matched docs, leaps, 1 if the segment's counts are unavailable:
 * a neighbour search of the fused count gave up) for every bound segment s of the last scan (synchronises `stream`). */
int32_t pa_query_leap_leaf(const pa_query* q);
int pa_query_leap_counts(pa_query* q, int64_t* out, void* stream);

/* Execution statistics of the DataTable (BaseResultsBlock.java:194 puts them in every results block):
 * numEntriesScannedInFilter / numEntriesScannedPostFilter of the bound segments after the last scan.
 *
 * The host passes the filter operator tree the reference builds for each segment (FilterPlanNode +
 * FilterOperatorUtils.getLeafFilterOperator / getAndFilterOperator / getOrFilterOperator: leaf operator choice from the
 * segment's indexes, constant children removed, AND children in reorderAndFilterChildOperators order), as pa_filter_op
 * nodes in pre-order; ops[tree_root[t] ..] is tree t. segment_tree[s] = the tree of bound segment s, or
 * PA_STATS_NON_SCAN (AggregationPlanNode's non-scan plans: neither count), PA_STATS_HOST (the host accounts for the
 * segment itself). The library derives what the reference's iterators read when the projection drives the tree's
 * iterator to the end (SVScanDocIdIterator / MVScanDocIdIterator next, advance and applyAnd; AndDocIdSet's merge of index
 * children; AndDocIdIterator's leap-frog, OrDocIdIterator, NotDocIdIterator) — constants, popcounts of applyAnd chains
 * and leap-frogs counted on the GPU over the segments' leaf bitmaps (pa_stats.hip) — or, when the scan counted a
 * two-scan AND itself (PA_QF_NO_FILTER_STATS unset), those counts.
 * out[0] = numEntriesScannedInFilter over the segments the library covered, out[1] = numEntriesScannedPostFilter =
 * (docs_scanned - docs of PA_STATS_NON_SCAN segments) x projected_columns (docs_scanned: numDocsScanned of the scan,
 * < 0 = the last scan's own counter), out[2] = segments whose count ran on the GPU. segment_in_filter[s]
 * (optional, host int64[num_segments]) = segment s's numEntriesScannedInFilter, or -1 for a segment the host must
 * account for (PA_STATS_HOST, or a tree shape outside the engine: a NOT child of a leap-frogging AND, an AND or NOT
 * child of an OR child of one). Synchronises `stream`. */
#define PA_FOP_EMPTY 0     /* EmptyFilterOperator */
#define PA_FOP_MATCH_ALL 1 /* MatchAllFilterOperator */
#define PA_FOP_SORTED 2    /* SortedIndexBasedFilterOperator (prog: its doc set) */
#define PA_FOP_BITMAP 3    /* BitmapBasedFilterOperator / RangeIndexBasedFilterOperator (exact) */
#define PA_FOP_SCAN 4      /* ScanBasedFilterOperator; mv_column >= 0: over that multi-value column */
#define PA_FOP_AND 5
#define PA_FOP_OR 6
#define PA_FOP_NOT 7
#define PA_STATS_NON_SCAN (-1)
#define PA_STATS_HOST (-2)
typedef struct {
  int32_t kind;          /* PA_FOP_* */
  int32_t num_children;  /* AND / OR: >= 2, NOT: 1, leaves: 0; the children follow in pre-order */
  int32_t mv_column;     /* PA_FOP_SCAN: column id of a multi-value column (-1: single-value) */
  int32_t prog_len;      /* leaves: the operator's doc set as a postfix program over the query's filter leaves */
  int32_t prog[PA_BIT_PROG_MAX];  /* (pa_bitmap_counts tokens) */
} pa_filter_op;
int pa_query_execution_stats(pa_query* q, int32_t num_ops, const pa_filter_op* ops, int32_t num_trees,
                             const int32_t* tree_root, const int32_t* segment_tree, int32_t projected_columns,
                             int64_t docs_scanned, int64_t* out, int64_t* segment_in_filter, void* stream);

/* Cross-GPU merge of hashed key spaces (parallel.merge_hashed_sections around one all-to-all). A row is one slot of
 * every per-key accumulator section (the numDocsScanned counters excluded) in section order: pa_query_row_bytes(q)
 * bytes; the packed key is one of its 8-byte units. pa_query_pack_rows writes the occupied slots (count > 0) as rows
 * grouped by the rank owning their key (a multiplicative hash of the packed key modulo `world`): counts[r] rows for
 * rank r, ranks in order, at device_rows (or, with device_rows NULL, only the counts). pa_query_merge_rows resets the
 * block and merges num_rows rows (from any rank holding the same key space) into it by packed key: SUM for counts
 * and sums, MIN, MAX, byte max for HLL registers and DISTINCTCOUNT presence (GroupByCombineOperator's merge);
 * *groups = the groups now held, *overflow = rows that found no free slot. Both synchronise `stream`. */
int64_t pa_query_row_bytes(const pa_query* q);
int pa_query_pack_rows(pa_query* q, int32_t world, void* device_rows, int64_t* counts, void* stream);
int pa_query_merge_rows(pa_query* q, const void* device_rows, int64_t num_rows, int64_t* groups, int64_t* overflow,
                        void* stream);

/* Group-key layout. Direct (hashed = 0): key = sum_j id_j * prod_{k<j} cardinality_k. Hashed (hashed = 1, chosen when
 * a group-by column is raw or the product of cardinalities is too large to address): the key packs component j
 * (a table-wide key id, or the raw value's bits: 32 for INT/FLOAT, 64 for LONG/DOUBLE) at bit shifts[j]; components
 * wider than 64 bits together take two key words (pa_query_key_words = 2: component j in word shifts[j] / 64 at bit
 * shifts[j] % 64, e.g. GROUP BY two raw LONG columns — NoDictionaryMultiColumnGroupKeyGenerator's composite keys), and
 * pa_query_fetch then writes two int64 per group into out_keys (out_keys holds 2 x capacity). Keys returned by
 * pa_query_fetch follow this layout. */
int pa_query_key_layout(const pa_query* q, int32_t* hashed, int32_t* shifts);
int32_t pa_query_key_words(const pa_query* q);

/* Kernel statistics of the last execute (for roofline accounting): bytes of forward index staged
 * (always-read columns), number of docs scanned. */
int pa_query_stats(const pa_query* q, uint64_t* staged_bytes, uint64_t* num_docs,
                   uint64_t* num_tiles);

/* The kernel plan chosen by pa_query_prepare: accumulator strategy (0 = LDS-privatised, 1 = global atomics,
 * 2 = partitioned: records partitioned by key range, then aggregated per partition in LDS; aggregation-only queries
 * 4..7 = per-lane register accumulators: 4 any column kinds, 5 COUNT only, 6 raw columns only, 7 dictionary
 * columns only; 8 = dense GROUP BY over a small key box, every column staged), 64-doc
 * steps per wave tile, DMA instructions per tile, tile images per wave, workgroups per CU, grid, LDS bytes. */
/* How the main scan pass reads a column (roofline byte model): 1 = staged (every word of every tile streamed through
 * LDS), 0 = read per surviving doc from HBM, -1 = the query does not read it in the main pass. */
int32_t pa_query_column_staged(const pa_query* q, int32_t column_id);
/* Filter literals evaluated on whole staged tiles (the rest only on the docs those matched). */
int32_t pa_query_num_eager_literals(const pa_query* q);
/* 1 if the lane-major scan kernel was chosen (lane l owns docs [32l, 32l+32) of a tile), 0 step-major, <0 error. */
int32_t pa_query_lane_major(const pa_query* q);
/* 1 if the dense GROUP BY kernel accumulates packed words (COUNT + every SUM term in one 64-bit LDS atomic per matching
 * doc, drained per wave into the workgroup's accumulators), 2 if it does so in the kernel specialised to the query's
 * shape (compiled by hiprtc at prepare), 0 if not, <0 error. */
int32_t pa_query_dense_packed(const pa_query* q);
/* 1 when the partitioned plan runs the count-free V emit (each workgroup writes whole record chunks into its own
 * region; pass C reads every partition through its chunk list: no count pass), 2 when it also runs the count-free H
 * emit (DISTINCTCOUNTHLLMV next to the V stream), 0 otherwise, <0 if not prepared. */
int32_t pa_query_count_free_emit(const pa_query* q);
/* Keys per partition of the partitioned plan's V stream (a power of two, or under the count-free emit any count that
 * spreads the key space over whole rounds of pass C's workgroups), 0 when the plan is not partitioned, <0 if not
 * prepared. */
int32_t pa_query_partition_keys(const pa_query* q);
int pa_query_plan(const pa_query* q, int32_t* strategy, int32_t* steps, int32_t* dma_slots, int32_t* ring,
                  int32_t* wg_per_cu, int32_t* grid, int32_t* lds_bytes);

void pa_query_destroy(pa_query* q);

#ifdef __cplusplus
}
#endif

#endif /* PINOT_AMD_H_ */
