/*
 * deequ_amd.h -- C ABI of the MI355X metric engine for deequ's metric-computation hot path.
 *
 * This is the drop-in boundary.  In the reference the hot path is reached
 * through two Scala/Spark contracts, both of which this ABI replaces:
 *
 *   (1) ScanShareableAnalyzer.aggregationFunctions(): Seq[Column] + fromAggregationResult(Row, offset)
 *       reference: src/main/scala/com/amazon/deequ/analyzers/Analyzer.scala:159-187, called once per
 *       suite by AnalysisRunner.runScanningAnalyzers (analyzers/runners/AnalysisRunner.scala:279-326,
 *       the single Spark job at :303).  -> dq_plan_create / dq_scan_device / dq_state_get
 *   (2) Spark's aggregate SPI that those Columns wrap (initialize / update / merge / eval):
 *       StatefulHyperloglogPlus.scala:74-146, StatefulStdDevPop.scala:24-34, StatefulCorrelation.scala:24-49
 *       and Spark's Count / Sum / Min / Max.  -> the per-row update runs in the HIP scan kernels,
 *       merge == dq_state_merge, eval == dq_state_get.
 *   (3) FrequencyBasedAnalyzer.computeFrequencies (analyzers/GroupingAnalyzers.scala:53-80) plus the
 *       one aggregation over the frequency table (AnalysisRunner.scala:466-534) and Histogram
 *       (analyzers/Histogram.scala:54-116).  -> dq_freq_* (hash group-by on the GPU).
 *
 * Conventions (mirroring the reference's): the caller owns every column buffer and keeps it alive
 * until dq_state_sync / dq_freq_summarize returns; the library never frees caller memory.  A plan is
 * immutable and may be shared between threads; a dq_state / dq_freq belongs to one thread (one
 * stream) at a time, like a Spark task's aggregation buffer.  No exception crosses this ABI: every
 * entry point returns a dq_status, and dq_last_error() returns the thread-local message of the
 * last failure (the host maps it to MetricCalculationRuntimeException, like
 * MetricCalculationException.wrapIfNecessary, runners/MetricCalculationException.scala:69-76).
 */
#ifndef DEEQU_AMD_H
#define DEEQU_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------------
 * Status codes
 * ---------------------------------------------------------------------------------------------- */
typedef enum dq_status {
  DQ_OK = 0,
  DQ_ERR_INVALID_ARGUMENT = 1, /* malformed plan / expression / argument                        */
  DQ_ERR_NO_SUCH_COLUMN = 2,   /* column index out of range (NoSuchColumnException)             */
  DQ_ERR_WRONG_TYPE = 3,       /* column type not valid for the aggregation (WrongColumnType...) */
  DQ_ERR_OUT_OF_MEMORY = 4,    /* device allocation failed                                      */
  DQ_ERR_DEVICE = 5,           /* HIP runtime error                                             */
  DQ_ERR_UNSUPPORTED = 6,      /* valid request outside what this engine implements             */
  DQ_ERR_STATE = 7             /* state / plan mismatch                                         */
} dq_status;

/* Thread-local message describing the last non-DQ_OK return on this thread. */
const char* dq_last_error(void);
/* ABI version (major*10000 + minor*100 + patch). */
int dq_version(void);
/* Number of HIP devices visible to this process (0 when there is no GPU). */
int dq_device_count(void);

/* ------------------------------------------------------------------------------------------------
 * Columns: Arrow-style buffers (Arrow columnar format, offset 0).
 * ---------------------------------------------------------------------------------------------- */
typedef enum dq_type {
  DQ_BOOL = 1,    /* Arrow "b": bit-packed values                                   */
  DQ_INT8 = 2,    /* "c" */
  DQ_INT16 = 3,   /* "s" */
  DQ_INT32 = 4,   /* "i" */
  DQ_INT64 = 5,   /* "l" */
  DQ_FLOAT32 = 6, /* "f" */
  DQ_FLOAT64 = 7, /* "g" */
  DQ_UTF8 = 8,    /* "u": int32 offsets (length+1) + bytes                           */
  /* Spark DecimalType(p, s) (Analyzer.scala:277-278, 322-327 count it numeric): Arrow "d:p,s"
   * (decimal128), 16-byte little-endian two's-complement unscaled values, 1 <= p <= 38,
   * 0 <= s <= p.  The type word carries p and s: DQ_DECIMAL_TYPE(p, s).                     */
  DQ_DECIMAL128 = 9,
  DQ_DATE32 = 10,      /* Spark DateType, Arrow "tdD": int32 days since 1970-01-01           */
  DQ_TIMESTAMP_US = 11 /* Spark TimestampType, Arrow "tsu:<tz>": int64 microseconds since
                          1970-01-01T00:00:00Z (text forms use UTC as the session time zone)  */
} dq_type;

/* A column type word: the dq_type in bits 0-7; for DQ_DECIMAL128 the precision in bits 8-15 and
 * the scale in bits 16-23 (a plan's column_types, dq_column.type and dq_freq key types all carry
 * the full word, so two decimal columns of different precision or scale are different types). */
#define DQ_TYPE_ID(t) ((int32_t)(t) & 0xff)
#define DQ_DECIMAL_TYPE(p, s) ((int32_t)DQ_DECIMAL128 | ((int32_t)(p) << 8) | ((int32_t)(s) << 16))
#define DQ_DECIMAL_PRECISION(t) (((int32_t)(t) >> 8) & 0xff)
#define DQ_DECIMAL_SCALE(t) (((int32_t)(t) >> 16) & 0xff)

typedef struct dq_column {
  int32_t type;            /* type word (dq_type, + precision / scale for DQ_DECIMAL128)     */
  int32_t data_bytes;      /* DQ_UTF8: optional size hint, >= offsets[length] - offsets[0] (the
                              group-by then sizes its key arena without reading the offsets
                              back); 0 = unknown.  Ignored for other types.                  */
  int64_t length;          /* rows                                                            */
  const uint8_t* validity; /* LSB-first bitmap (1 = valid), NULL when the column has no nulls */
  const void* values;      /* fixed-width values; for DQ_UTF8 the int32 offsets               */
  const uint8_t* data;     /* DQ_UTF8 character bytes, otherwise NULL                         */
} dq_column;

/* Arrow C Data Interface (https://arrow.apache.org/docs/format/CDataInterface.html), verbatim. */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif

/* Converts one Arrow C Data Interface array (primitive or utf8, any offset) into a dq_column that
 * aliases the same buffers.  The JNI shim calls this on each exported
 * DataFrame-partition column (a sliced partition carries a non-zero ArrowArray.offset).  Values and
 * utf8 offsets are aliased at the slice's first row (utf8 offsets stay absolute into the character
 * buffer); a validity bitmap (or boolean values) whose offset is not a whole number of bytes is
 * copied, re-based to bit 0, into the memory space it came from (device or host), and owned by the
 * library until dq_column_release.  Buffers may be host or device pointers; the caller says which
 * by the entry point it hands the column to. */
dq_status dq_column_from_arrow(const struct ArrowArray* array, const struct ArrowSchema* schema,
                               dq_column* out);
/* Frees what dq_column_from_arrow allocated for `col` (re-based bitmaps); a no-op for a column
 * that only aliases Arrow buffers. */
void dq_column_release(dq_column* col);

/* ------------------------------------------------------------------------------------------------
 * Expressions (SQL predicates of `where` filters and Compliance / Check constraints).
 *
 * An expression is a prefix-order sequence of int64 words.  The host compiles deequ's SQL strings
 * (Check.scala:538-548, 670-760, 826-869; Analyzers.conditionalSelection Analyzer.scala:385-408)
 * into it after Spark-2.2 type coercion, so the engine only sees typed operations.  Evaluation uses
 * SQL three-valued logic (TRUE / FALSE / NULL) exactly like Catalyst.
 * ---------------------------------------------------------------------------------------------- */
typedef enum dq_xop {
  DQ_X_COL = 1,        /* [op, column]                      value of a column                    */
  DQ_X_NULL = 2,       /* [op]                              NULL literal                         */
  DQ_X_BOOL = 3,       /* [op, 0|1]                         boolean literal                      */
  DQ_X_I64 = 4,        /* [op, value]                       integral literal                     */
  DQ_X_F64 = 5,        /* [op, bits]                        double literal (IEEE bits)           */
  DQ_X_STR = 6,        /* [op, nbytes, ceil(n/8) words]     UTF-8 literal, little-endian packed  */
  DQ_X_IS_NULL = 7,    /* [op, x]                                                                */
  DQ_X_IS_NOT_NULL = 8,/* [op, x]                                                                */
  DQ_X_NOT = 9,        /* [op, x]                                                                */
  DQ_X_AND = 10,       /* [op, a, b]                        Kleene AND                           */
  DQ_X_OR = 11,        /* [op, a, b]                        Kleene OR                            */
  DQ_X_EQ = 12,        /* [op, a, b]  comparisons: numeric operands compared after promotion to  */
  DQ_X_NE = 13,        /*             the wider type (double compare is Spark's NaN-safe order), */
  DQ_X_LT = 14,        /*             strings compared bytewise (UTF8String.compareTo)           */
  DQ_X_LE = 15,
  DQ_X_GT = 16,
  DQ_X_GE = 17,
  DQ_X_EQ_NULL_SAFE = 18, /* <=> */
  DQ_X_IN = 19,        /* [op, n, x, item_1 .. item_n]      x IN (items)                          */
  DQ_X_CAST_F64 = 20,  /* [op, x]                           CAST(x AS DOUBLE) (string: parse); a  */
                       /*   float32 value is widened exactly and prints as Double.toString after */
  DQ_X_REGEX = 21,     /* [op, null_mode, nbytes, ceil(n/8) words, x]  regex find() over x's text:
                          the words pack an automaton (deequ_amd/regex.py CompiledRegex.blob):
                          int32 n_states, n_classes, start, 0; u8 byte_class[256]; u8
                          status[n_states] (1 accept, 2 reject, padded to 4); u16
                          next[n_states * n_classes], the last class being end-of-text.  x is
                          a string (integral / boolean x are formatted as Spark's cast to
                          string).  A NULL x gives NULL (null_mode 0, RLIKE) or FALSE
                          (null_mode 1: when(regexp_extract(x, p, 0) != "", 1).otherwise(0),
                          PatternMatch.scala:44-46).                                           */
  DQ_X_CAST_F32 = 22,  /* [op, x]  CAST(x AS FLOAT): an integral x rounds to the nearest float,
                          a double one too (Spark's Cast to FloatType, `.toFloat`); the value
                          then prints as Float.toString.  A string x (utf8 column or literal)
                          is refused by dq_plan_create with DQ_ERR_UNSUPPORTED:
                          Float.parseFloat's direct rounding is not restated.                  */
  DQ_X_DEC128 = 23     /* [op, lo, hi]  decimal literal as an unscaled 128-bit value at the scale of
                          the DQ_DECIMAL128 column it is compared with (the host rescales it, so
                          the comparison is exact, as Spark's DecimalPrecision makes it).  A
                          decimal column may appear under IS [NOT] NULL, in comparisons / IN with
                          DQ_X_DEC128 items, under DQ_X_CAST_F64 (Decimal.toDouble, correctly
                          rounded) and as a regex operand (BigDecimal.toString text); a date /
                          timestamp column under IS [NOT] NULL and as a regex operand.  Any other
                          use is refused by dq_plan_create with DQ_ERR_UNSUPPORTED.            */
} dq_xop;

typedef struct dq_expr {
  const int64_t* words;
  int32_t n_words;
  int32_t reserved;
} dq_expr;

/* ------------------------------------------------------------------------------------------------
 * Scan plan: the concatenated aggregation functions of every ScanShareableAnalyzer of a suite, in
 * analyzer order, exactly as AnalysisRunner builds `aggregations` and their `offsets`
 * (AnalysisRunner.scala:296-301).  One dq_agg == one Column of aggregationFunctions().
 * ---------------------------------------------------------------------------------------------- */
typedef enum dq_agg_kind {
  DQ_AGG_COUNT_ALL = 1,     /* count("*")                                   Size / Mean / ratios   */
  DQ_AGG_COUNT_NOTNULL = 2, /* sum(isNotNull(when(where, col)).cast(Int))   Completeness.scala:44  */
  DQ_AGG_COUNT_TRUE = 3,    /* sum(when(where, expr).cast(Int|Long))        Compliance.scala:48,
                                                                            conditionalCount :404  */
  DQ_AGG_SUM = 4,           /* sum(when(where, col))                        Sum.scala:35, Mean:39  */
  DQ_AGG_MIN = 5,           /* min(when(where, col))                        Minimum.scala:36       */
  DQ_AGG_MAX = 6,           /* max(when(where, col))                        Maximum.scala:36       */
  DQ_AGG_STDDEV_POP = 7,    /* stateful_stddev_pop(when(where, col))        StandardDeviation:49   */
  DQ_AGG_CORR = 8,          /* stateful_corr(when(where,x), when(where,y))  Correlation.scala:81   */
  DQ_AGG_HLL = 9,           /* stateful_approx_count_distinct(...)          ApproxCountDistinct:43 */
  DQ_AGG_DTYPE = 10         /* stateful_datatype(when(where, col))           DataType.scala:171-173:
                               words[0..4] = NULL, Fractional, Integral, Boolean, String counts   */
} dq_agg_kind;

typedef struct dq_agg {
  int32_t kind;  /* dq_agg_kind                                           */
  int32_t col;   /* input column (-1 for COUNT_ALL / COUNT_TRUE)          */
  int32_t col2;  /* second column (CORR), else -1                         */
  int32_t expr;  /* COUNT_TRUE: index of the counted expression, else -1  */
  int32_t where; /* index of the `where` expression, -1 for none          */
  int32_t reserved;
} dq_agg;

typedef struct dq_plan_desc {
  int32_t n_columns;
  const int32_t* column_types; /* dq_type per column index (the schema) */
  int32_t n_exprs;
  const dq_expr* exprs;
  int32_t n_aggs;
  const dq_agg* aggs;
} dq_plan_desc;

typedef struct dq_plan dq_plan;
dq_status dq_plan_create(const dq_plan_desc* desc, dq_plan** out);
void dq_plan_destroy(dq_plan* plan);
/* Human-readable listing of the fused tasks the planner produced (for tests / EXPLAIN). */
dq_status dq_plan_explain(const dq_plan* plan, char* buf, size_t buf_len);
/* Number of kernel launches one dq_scan_device call issues for this plan (the analogue of the
 * reference's Spark-job-count assertions, AnalysisRunnerTests.scala:34-102). */
int dq_plan_launches_per_batch(const dq_plan* plan);

/* ------------------------------------------------------------------------------------------------
 * Aggregation state: per-agg partial states, device resident while scanning.
 * ---------------------------------------------------------------------------------------------- */
typedef struct dq_state dq_state;
/* device = -1 creates a host-only state (no GPU needed) that supports reset / deserialize /
 * merge / get / serialize: the rank-ordered merge after a multi-GPU all-gather uses it. */
dq_status dq_state_create(const dq_plan* plan, int device, dq_state** out);
void dq_state_destroy(dq_state* state);
dq_status dq_state_reset(dq_state* state);

/* Scans one batch of rows whose buffers live in device memory.  Stream-ordered on `hip_stream`
 * (a hipStream_t, NULL = default stream); results accumulate into `state` across batches like
 * Spark partial aggregation over partitions.  cols[i] must match the plan schema. */
dq_status dq_scan_device(const dq_plan* plan, const dq_column* cols, int n_cols, dq_state* state,
                         void* hip_stream);
/* Scans `n_batches` device-resident batches (cols is [n_batches][n_cols], row-major) in ONE fused
 * launch: a DataFrame held as several Arrow record batches (int32 string offsets cap a batch at
 * 2 GiB of characters) is still a single pass, like the reference's single Spark job. */
dq_status dq_scan_device_batches(const dq_plan* plan, const dq_column* cols, int n_cols,
                                 int n_batches, dq_state* state, void* hip_stream);
/* Waits for the state's stream and finalises the slot values on the host. */
dq_status dq_state_sync(dq_state* state);

/* One typed aggregation result (one slot of the reference's result Row).
 *   COUNT_*  : i64 (is_null per Spark: a sum over no non-null input is NULL)
 *   SUM      : integral input: i64 = wrapping Long sum, f64[0] = (double)i64; floating: f64[0];
 *              decimal(p, s): words[0..3] = the exact sum of the unscaled values (256-bit two's
 *              complement, little-endian words), f64[0] = Cast(sum AS DOUBLE) correctly rounded;
 *              is_null also when the sum does not fit Spark 2.2's result type
 *              decimal(min(p + 10, 38), s) (Sum.scala:35 over Spark's Sum)
 *   MIN/MAX  : f64[0] (= cast of the native-typed extreme); i64 = the native integral extreme;
 *              decimal: words[0..1] = the unscaled 128-bit extreme, f64[0] its correctly rounded
 *              cast
 *   STDDEV   : f64[0..2] = n, avg, m2 (never NULL; n == 0 means no input); a decimal column's
 *              values enter as their cast to double (CentralMomentAgg's DoubleType input)
 *   CORR     : f64[0..5] = n, xAvg, yAvg, ck, xMk, yMk
 *   HLL      : words[0..51] = the 52 register words in reference order (never NULL)      */
typedef struct dq_value {
  int32_t kind;
  int32_t is_null;
  int64_t i64;
  double f64[6];
  uint64_t words[52];
} dq_value;
dq_status dq_state_get(const dq_state* state, int agg_index, dq_value* out);
/* dq_state_get for aggregations 0 .. n-1 into out[0 .. n-1] in one call (the per-step result
 * read-out of a scan: one foreign call instead of one per aggregation). */
dq_status dq_state_get_all(const dq_state* state, int n, dq_value* out);

/* dst += src for two synced states of one plan: Spark's partial-aggregation merge of every
 * aggregation buffer -- what happens between the partitions of ONE Spark job, and here between
 * batches, workgroups and GPU ranks: counts add (a NULL sum is the identity), Long sums wrap,
 * Min/Max in Spark's NaN-safe order, (n, avg, m2) per CentralMomentAgg merge ==
 * StandardDeviationState.sum (StandardDeviation.scala:37-44), co-moments per Corr merge ==
 * CorrelationState.sum (Correlation.scala:37-52), HLL register max (StatefulHyperloglogPlus.scala:
 * 119-137).  deequ's analyzer-level State.sum (incremental runs) lives on the host side. */
dq_status dq_state_merge(dq_state* dst, const dq_state* src);
/* Fixed-size little-endian image of the synced slot values (for collectives / persistence). */
int64_t dq_state_serialized_size(const dq_plan* plan);
dq_status dq_state_serialize(const dq_state* state, void* buf, int64_t buf_len);
dq_status dq_state_deserialize(dq_state* state, const void* buf, int64_t buf_len);

/* State exchange across ranks, on the device (distributed.py exchange_states):
 * the merge Spark performs over partition states (Analyzer.scala:337-362 / StateLoader) split
 * into the collectives each field's merge rule allows:
 *   isum[n_sum]   int64, all-reduce SUM: every task's counters and wrapping Long sums, the rows;
 *   imax[n_max]   int64, all-reduce MAX: max keys, bitwise-NOT min keys (MAX of ~x = ~MIN);
 *   hll[n_hll]    uint8, all-reduce MAX: the HLL registers (StatefulHyperloglogPlus.scala:119-137
 *                 merges by max);
 *   mom[n_mom]    double, all-GATHER (rank-major [world][n_mom]): n and the fp64 moments, merged
 *                 in rank order by the Chan / co-moment rules (StandardDeviation.scala:37-44,
 *                 Correlation.scala:37-52), and a decimal task's exact 192-bit sum and 128-bit
 *                 extremes as raw words (merged in the same rank-ordered pass).
 * pack fills the four buffers from the state (device pointers for a device state: a kernel on the
 * state's stream that hip_stream is made to wait for; host pointers for a host state, device
 * -1); unpack writes the merged result into the state (device: a kernel on the state's stream
 * after hip_stream; read it with dq_state_sync).  Neither waits on the host (the plan's task kinds
 * reach the device once per state).  The result equals dq_state_merge over the ranks' states in
 * rank order, byte for byte. */
dq_status dq_state_exchange_sizes(const dq_plan* plan, int64_t* n_sum, int64_t* n_max,
                                  int64_t* n_mom, int64_t* n_hll);
dq_status dq_state_exchange_pack(dq_state* state, int64_t* isum, int64_t* imax, double* mom,
                                 uint8_t* hll, void* hip_stream);
dq_status dq_state_exchange_unpack(dq_state* state, const int64_t* isum, const int64_t* imax,
                                   const double* mom_gathered, const uint8_t* hll, int world,
                                   void* hip_stream);
/* Host waits on device work (stream / event synchronisations) the state and scan entry points
 * have made in this process: a diagnostic counter (tests assert a path's waits, e.g. one per state
 * exchange -- the merged state's read-back). */
int64_t dq_host_wait_count(void);

/* HyperLogLogPlusPlusUtils.count (StatefulHyperloglogPlus.scala:208-255) on 52 register words.
 * `bias_corrected` is set to 1 when the estimate fell in the empirical-bias range (E < 5M with no
 * linear counting); that branch needs Spark's RAW_ESTIMATE_DATA/BIAS_DATA tables, which are not
 * available here, so the raw estimate is returned there (documented parity gap). */
double dq_hll_count(const uint64_t* words, int* bias_corrected);
/* Spark XxHash64Function.hash(v, type, 42) for one value (host reference of the device hash). */
uint64_t dq_xxhash64(const void* data, int64_t nbytes, uint64_t seed);
/* Java's Double.toString / Float.toString of one value (Spark 2.2 Cast(Double|FloatType ->
 * StringType), the text PatternMatch.scala:44-48 and Histogram.scala:59-66 see for a floating-point
 * column): the device formatter of jfmt.h, run on the host.  Writes at most 26 bytes, no NUL;
 * returns the length. */
int dq_java_double_to_string(double value, char* buf);
int dq_java_float_to_string(float value, char* buf);
/* The same for n values at once (Histogram's keys of a floating-point column): value i's text at
 * out + 32 i, its length in lens[i]; is_float: Float.toString of (float) values[i]. */
void dq_java_doubles_to_strings(const double* values, int64_t n, int is_float, char* out,
                                int32_t* lens);
/* Spark's Cast(DecimalType(p, s) AS DOUBLE) (Decimal.toDouble = java.math.BigDecimal.doubleValue:
 * the double nearest to unscaled / 10^s, ties to even) of one 128-bit unscaled value given as its
 * low and high words: the device conversion (decimal.h) run on the host. */
double dq_decimal_to_double(uint64_t lo, int64_t hi, int32_t scale);
/* Spark 2.2's Cast(x AS STRING) of n values of a DQ_DECIMAL128 / DQ_DATE32 / DQ_TIMESTAMP_US
 * column (`type` = its type word, values as the column stores them): java.math.BigDecimal
 * .toString (plain, or E-notation when the adjusted exponent is below -6), "yyyy-MM-dd"
 * (DateTimeUtils.dateToString) and "yyyy-MM-dd HH:mm:ss[.fraction]" in UTC
 * (DateTimeUtils.timestampToString; the fraction is the nanoseconds without trailing zeros).
 * Value i's text at out + 64 i (no NUL), its length in lens[i].  Histogram's keys of such a column
 * (Histogram.scala:63); the device formats the same text for PatternMatch (dtfmt.h). */
dq_status dq_format_values(int32_t type, const void* values, int64_t n, char* out, int32_t* lens);

/* ------------------------------------------------------------------------------------------------
 * Frequency path: hash group-by (FrequencyBasedAnalyzer.computeFrequencies) on the GPU.
 * ---------------------------------------------------------------------------------------------- */
typedef struct dq_freq dq_freq;

/* Creates an empty frequency table for grouping on `n_keys` columns of the given types.
 * `capacity_hint` is the expected number of distinct groups (0 = unknown). */
dq_status dq_freq_create(int device, int n_keys, const int32_t* key_types, int64_t capacity_hint,
                         dq_freq** out);
void dq_freq_destroy(dq_freq* freq);
/* Empties the table (groups, counters, numRows) and keeps its device capacity, stream-ordered on
 * `hip_stream`.  Replaces re-creating the per-task aggregation buffer of the grouping job
 * (GroupingAnalyzers.scala:70, a fresh HashAggregate buffer per task). */
dq_status dq_freq_reset(dq_freq* freq, void* hip_stream);
/* Inserts one batch: rows where any key is NULL are skipped but counted in numRows
 * (GroupingAnalyzers.scala:62-77).  Histogram mode (null_as_group != 0, one key column) instead
 * counts the NULL rows as one group kept apart from every keyed group (export / top-k report it
 * with tag 0); na.fill("NullValue") (Histogram.scala:59-66) folds it into a "NullValue" string
 * group, which the caller does with dq_freq_null_literal.  Kept apart, the same table also serves
 * the column's grouping (dq_freq_summarize_keys). */
dq_status dq_freq_add_device(dq_freq* freq, const dq_column* keys, int n_keys, int null_as_group,
                             void* hip_stream);

/* One aggregation over the frequency table (AnalysisRunner.scala:490-500):
 *   n_unique  = Σ[count == 1]    (Uniqueness.scala:29, UniqueValueRatio.scala:28)
 *   n_groups  = count(*)         (CountDistinct.scala:27, Distinctness via Σ[count >= 1])
 *   entropy   = Σ −(c/numRows)·ln(c/numRows)   (Entropy.scala:33-40)
 *   num_rows  = rows added, nulls included (data.count()) */
typedef struct dq_freq_summary {
  int64_t num_rows;
  int64_t n_groups;
  int64_t n_unique;
  int64_t n_null_key_rows;
  double entropy;
} dq_freq_summary;
dq_status dq_freq_summarize(dq_freq* freq, dq_freq_summary* out);
/* The same aggregation over the keyed groups only: a table built with NULL as a group
 * (Histogram mode) summarised as the grouping of that column would be, its NULL rows dropped
 * (GroupingAnalyzers.scala:62-65).  Lets one group-by serve Histogram(col) and the
 * Uniqueness/Distinctness/Entropy grouping of col.  n_null_key_rows counts the NULL rows. */
dq_status dq_freq_summarize_keys(dq_freq* freq, dq_freq_summary* out);

/* The marginal of key column key_index of a multi-key grouping table, added into `out` (a table
 * with one key of that column's type): every group of `joint` contributes its count to the group
 * of its key_index value, and out's numRows grows by joint's.  MutualInformation
 * (MutualInformation.scala:41-70) needs these marginals of the joint frequencies. */
dq_status dq_freq_marginal(dq_freq* joint, int key_index, dq_freq* out, void* hip_stream);

/* MutualInformation (MutualInformation.scala:41-84) of a two-key grouping table: the sum over its
 * groups of (pxy/n) ln((pxy/n) / ((px/n)(py/n))), n = numRows, px / py the marginal counts
 * (re-aggregated from the joint table on the device and joined by key).  *is_null = 1 when the
 * table has no groups (the reference's sum is then NULL -> empty state). */
dq_status dq_freq_mutual_information(dq_freq* joint, double* mi, int* is_null, void* hip_stream);

/* ApproxCountDistinct's 52 register words (StatefulHyperloglogPlus.scala:87-113 layout) from a
 * one-column table's partitioned records, when it holds at most max_records of them: the
 * registers depend only on the set of distinct non-NULL values, so a table already built for a
 * grouping or Histogram of the column yields them without a pass over the rows (its records are
 * fewer than the rows once repeated keys collapsed).  *done = 0 (words untouched) when the table
 * has more records, or is not a one-column fixed-width / utf8 table; the caller then scans. */
dq_status dq_freq_hll(dq_freq* table, int64_t max_records, uint64_t* words, int* done,
                      void* hip_stream);

/* Keyed rows of a Histogram-mode floating-point table (null_as_group) whose NaN payload was folded
 * into the canonical NaN -- Histogram groups cast(col as string), where every NaN prints "NaN"
 * (Histogram.scala:63), while a grouping keeps Spark 2.2's binary key equality.  0: the table's
 * keyed groups are exactly the grouping's of the same column (the runner then groups the column
 * once); -1: not counted (a batch took a path that does not count, or records were merged in). */
dq_status dq_freq_folded_nan_rows(dq_freq* table, int64_t* n);

/* Number of groups currently in the table (NULL group and every distinct key). */
dq_status dq_freq_num_groups(dq_freq* freq, int64_t* n_groups);
/* Histogram's NULL fold (Histogram.scala:59-66, na.fill("NullValue") before the groupBy): the rows
 * of the NULL group, and the count of the string group "NullValue" of a one-utf8-key Histogram
 * table (0 for every other table).  Histogram's group "NullValue" has their sum as its count;
 * numberOfBins is dq_freq_num_groups minus 1 when both are non-zero. */
dq_status dq_freq_null_literal(dq_freq* freq, int64_t* null_group_rows, int64_t* literal_count);
/* Rows added so far (nulls included): the numRows of FrequenciesAndNumRows. */
int64_t dq_freq_num_rows(const dq_freq* freq);
/* Exports every group (unordered): counts_out[n], key_offsets_out[n + 1] and the encoded keys:
 * per key column a u32 tag (0 = NULL, 1 = value) followed by 8 little-endian value bytes (the
 * value widened to 64 bits: integers sign-extended, float/double as their IEEE bits) or, for
 * utf8, a u32 byte length and the bytes padded to a multiple of 4.  Call with key_bytes_out = NULL
 * to learn the sizes (*key_bytes_needed, and dq_freq_num_groups for n). */
dq_status dq_freq_export(dq_freq* freq, int64_t* counts_out, int64_t* key_offsets_out,
                         uint8_t* key_bytes_out, int64_t capacity, int64_t key_bytes_capacity,
                         int64_t* key_bytes_needed);
/* The k groups with the largest counts, in descending count order (ties in any order), in the
 * export format: Histogram's details, rdd.top(maxDetailBins)(OrderByAbsoluteCount)
 * (Histogram.scala:78-79; numberOfBins is dq_freq_num_groups; see dq_freq_null_literal for the
 * NULL fold of a string column).  Only these k keys leave the
 * device.  Call with key_bytes_out = NULL for *n_out and *key_bytes_needed; counts_out[k] and
 * key_offsets_out[k + 1] must hold k entries. */
dq_status dq_freq_topk(dq_freq* freq, int k, int64_t* counts_out, int64_t* key_offsets_out,
                       uint8_t* key_bytes_out, int64_t key_bytes_capacity, int64_t* n_out,
                       int64_t* key_bytes_needed);
/* dst += src: the null-safe full-outer-join merge of two frequency states
 * (FrequenciesAndNumRows.sum, GroupingAnalyzers.scala:128-148): counts of equal keys add and
 * numRows add.  Keys are compared as encoded keys, so a 64-bit hash collision between the two
 * tables' groups never merges them. */
dq_status dq_freq_merge(dq_freq* dst, const dq_freq* src);

/* ------------------------------------------------------------------------------------------------
 * Multi-GPU frequency path: hash repartition.
 *
 * Replaces the hash-partitioned Exchange between Spark's partial and final HashAggregate of the
 * groupBy in computeFrequencies (GroupingAnalyzers.scala:67-72).  Each rank's table is the partial
 * aggregate of its row shard.  dq_freq_partition cuts its groups into n_parts owner segments
 * (owner = a hash of the group key, so every group has exactly one owner); the caller exchanges
 * the segments with an all-to-all (RCCL over xGMI) and each owner re-inserts what it received with
 * dq_freq_add_records_device, which adds counts of equal keys exactly like FrequenciesAndNumRows.sum
 * (GroupingAnalyzers.scala:128-148).  Records are device memory; var holds the encoded keys of
 * hashed-mode tables (string / multi-column keys), 8-byte aligned per group.
 * ---------------------------------------------------------------------------------------------- */
typedef struct dq_freq_record {
  uint64_t key;     /* exact mode (one fixed-width key): the widened key value; hashed mode
                       (strings / several keys / Histogram on strings): the 64-bit group hash      */
  uint64_t count;   /* rows in the group                                                          */
  uint64_t enc_off; /* hashed mode: byte offset of the encoded key within the segment's var bytes */
} dq_freq_record;
/* Per owner: rec_counts[n_parts] records and var_bytes[n_parts] bytes.  special[3] = the counts
 * kept outside the records, which the caller routes to ONE owner: {0 (unused), rows of the
 * NULL group (Histogram), rows skipped for a NULL key}. */
dq_status dq_freq_partition_sizes(dq_freq* freq, int n_parts, int64_t* rec_counts,
                                  int64_t* var_bytes, int64_t* special);
/* Writes the owner segments back to back (segment j at the exclusive prefix sums of the sizes
 * above) into device buffers records[Σ rec_counts] and var[Σ var_bytes]. */
dq_status dq_freq_partition(dq_freq* freq, int n_parts, dq_freq_record* records, uint8_t* var,
                            void* hip_stream);
/* Inserts n_src received segments laid back to back (src_records[j] records, src_var_bytes[j]
 * var bytes each), adds num_rows to the table's numRows and special[3] to its outside-record
 * counts.  Groups with equal keys add their counts; equal hashes with different encoded keys stay
 * separate groups. */
dq_status dq_freq_add_records_device(dq_freq* freq, const dq_freq_record* records,
                                     const uint8_t* var, int n_src, const int64_t* src_records,
                                     const int64_t* src_var_bytes, int64_t num_rows,
                                     const int64_t* special, int null_as_group, void* hip_stream);

/* Raw-key repartition (the same Exchange, for a one-column fixed-width key of high cardinality:
 * int8..int64, float, double).  Exchanging the rows' raw values before any local count costs one
 * group-by per row on the owner and 1-8 bytes per row over the link, where partitioning a partial
 * table costs a group-by on every rank, 24-byte records and a second group-by.  Writes the non-NULL
 * values of all batches into out (device, (rows of all batches) x element size bytes), owner j's
 * segment at the exclusive prefix of counts_out[0..n_parts); the owner is a function of the key the
 * table counts (NaN payloads canonical under null_as_group, as in dq_freq_add_device), so equal
 * keys of every rank meet on one owner.  NULL rows stay home: *null_rows_out.  Synchronous. */
dq_status dq_key_partition(const dq_column* batches, int n_batches, int n_parts, int null_as_group,
                           uint8_t* out, int64_t* counts_out, int64_t* null_rows_out,
                           void* hip_stream);

/* Returns the device blocks the engine keeps cached for reuse (every dq_* buffer is handed back
 * to a per-device cache when freed, so building many tables does not hipMalloc / hipFree
 * gigabytes each time) to the HIP runtime. */
void dq_release_cached_memory(void);

/* Bytes of idle device blocks the engine's cache holds for `device` (reusable by the next dq_*
 * allocation without a hipMalloc; the runner adds them to hipMemGetInfo's free bytes when it
 * decides whether two group-by tables may be on the device at once).  No reference counterpart:
 * Spark's memory manager is the JVM's. */
int64_t dq_cached_device_bytes(int device);

/* Spark 2.2 Cast(StringType -> LongType | DoubleType) of a utf8 column, on the device: the
 * ColumnProfiler's cast of string columns inferred numeric (profiles/ColumnProfiler.scala:311-320,
 * 389-405).  to_type DQ_INT64 follows UTF8String.toLong (sign, digits, '.' + digits truncated);
 * DQ_FLOAT64 follows java.lang.Double.parseDouble over decimal strings.  A string that does not
 * convert is NULL in validity_out (LSB-first, (length + 7) / 8 bytes); values_out holds length
 * int64 / double.  *n_unsupported counts strings parseDouble would read that are not converted
 * here exactly (exponents, NaN/Infinity, hex, > 19 significant digits ...): those rows are NULL and
 * the caller must treat a non-zero count as a failure.  Synchronises `hip_stream`. */
dq_status dq_cast_utf8(const dq_column* in, int to_type, void* values_out, uint8_t* validity_out,
                       int64_t* n_unsupported, void* hip_stream);

/* ------------------------------------------------------------------------------------------------
 * Columnar handoff: host-resident Arrow batches -> HBM (the JNI shim's entry).
 *
 * In the reference a Spark partition's rows stream through the aggregation iterator of the one
 * `data.agg(...)` job (AnalysisRunner.scala:303) and of the grouping job
 * (GroupingAnalyzers.scala:62-77).  Here a partition arrives as host Arrow buffers
 * (dq_column_from_arrow), is copied into one of two pinned staging buffers (host threads), DMA'd
 * into the slot's device buffer on the loader's copy stream, and scanned on the caller's stream;
 * the DMA of batch k+1 overlaps the scan of batch k.  Lifetime: the loader reads the caller's host
 * buffers only inside dq_loader_stage / dq_scan_host / dq_freq_add_host -- they may be freed or
 * reused as soon as the call returns (unlike the device entry points' buffers, which must stay
 * valid until dq_state_sync / dq_freq_summarize).  One loader per thread / stream, like a
 * dq_state.
 * ---------------------------------------------------------------------------------------------- */
typedef struct dq_loader dq_loader;
dq_status dq_loader_create(int device, dq_loader** out);
void dq_loader_destroy(dq_loader* loader);
/* Stages one host batch: copies it into the slot's pinned buffer, enqueues the DMA and makes
 * `hip_stream` wait for it; writes the
 * device-pointer columns to dev_cols[n_cols].  Every staged batch must be released (below) after
 * the work that reads dev_cols has been enqueued on `hip_stream`. */
dq_status dq_loader_stage(dq_loader* loader, const dq_column* host_cols, int n_cols,
                          dq_column* dev_cols, void* hip_stream);
dq_status dq_loader_release(dq_loader* loader, void* hip_stream);
/* stage + dq_scan_device + release. */
dq_status dq_scan_host(dq_loader* loader, const dq_plan* plan, const dq_column* host_cols,
                       int n_cols, dq_state* state, void* hip_stream);
/* stage + dq_freq_add_device + release. */
dq_status dq_freq_add_host(dq_loader* loader, dq_freq* freq, const dq_column* host_keys, int n_keys,
                           int null_as_group, void* hip_stream);

/* ------------------------------------------------------------------------------------------------
 * ApproxQuantile (ApproxQuantile.scala:41-104): the device sorts the non-NULL values of a numeric
 * column (all batches, cast to double as ApproximatePercentile does; NaNs canonical, so the order
 * is Java's Double.compare) and returns either every value (when count <= head_values; the host
 * then replays Spark's QuantileSummaries exactly) or max_values of them at the exact ranks
 * floor(j * (count - 1) / (max_values - 1)).  out holds max(head_values, max_values) doubles (host
 * memory; min(..., rows) suffices); *n_out = values written, *count_out = non-NULL values.
 * Synchronous on hip_stream.
 * ---------------------------------------------------------------------------------------------- */
dq_status dq_sorted_sample(int device, const dq_column* batches, int n_batches, int64_t head_values,
                           int64_t max_values, double* out, int64_t* n_out, int64_t* count_out,
                           void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* DEEQU_AMD_H */
