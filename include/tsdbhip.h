/*
 * tsdbhip.h — C-ABI of libtsdbhip.so, the MI355X (gfx950) query-time
 * aggregation path of OpenTSDB 1.1 (reference: anonthing/opentsdb).
 *
 * Plain pointers and sizes only; no HIP, torch or C++ types cross this
 * boundary, so the Java host binds it through a thin JNI shim (see
 * INTEGRATION.md) and Python through ctypes (opentsdb_amd/_lib.py).
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference root):
 *
 *   tsdbhip_spangroup_run  — the whole lazy iteration of a SpanGroup as the
 *       consumers drive it (GraphHandler.java:791-808, Plot.java:190-204,
 *       CliQuery.java:161-170): SpanGroup ctor/add (SpanGroup.java:104-142),
 *       SGIterator (SpanGroup.java:370-796), Span.Iterator /
 *       Span.DownsamplingIterator (Span.java:248-530), RowSeq.Iterator
 *       (RowSeq.java:360-497) and the five Aggregators (Aggregators.java:76-243).
 *       Row assembly follows Span.addRow / RowSeq.addRow (Span.java:87-132,
 *       RowSeq.java:92-172), i.e. what TsdbQuery.findSpans does with each
 *       compacted KeyValue (TsdbQuery.java:240-285).
 *   tsdbhip_spangroup_run_batch — the SpanGroup[] of a GROUP BY query
 *       (TsdbQuery.groupByAndAggregate, TsdbQuery.java:294-363), all groups in
 *       one call.
 *   tsdbhip_format_points  — the text GraphHandler.respondAsciiQuery,
 *       Plot.dumpToFiles and CliQuery print for each DataPoint.
 *   tsdbhip_compact_rows   — CompactionQueue.compact(row, compacted[])
 *       (CompactionQueue.java:243-435, 450-743) for a batch of rows.
 *   tsdbhip_host_register / unregister — pinning of the JNI DirectByteBuffers
 *       the bridge packs at TsdbQuery.java:264-266.
 *
 * Errors map to the reference's exceptions (the JNI shim rethrows them):
 *   TSDBHIP_E_ILLEGAL_DATA -> IllegalDataException   (RowSeq.java:203,223;
 *                             CompactionQueue.java:324,538,640,717,736)
 *   TSDBHIP_E_NAN_INF      -> IllegalStateException  (SpanGroup.java:660-663)
 *   TSDBHIP_E_EMPTY_SPAN   -> AssertionError         (SpanGroup.java:452-455)
 *   others                 -> RuntimeException
 * The reference is lazy (exceptions surface while iterating); this library
 * is eager. out->err_index carries the index of the first output point the
 * reference would NOT have delivered (-1 when unknown), so a host adapter can
 * replay the lazy behaviour.
 */
#ifndef TSDBHIP_H
#define TSDBHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSDBHIP_ABI_VERSION 7

/* ---- return codes ---------------------------------------------------- */
#define TSDBHIP_OK               0
#define TSDBHIP_E_ILLEGAL_DATA  -1
#define TSDBHIP_E_NAN_INF       -2
#define TSDBHIP_E_EMPTY_SPAN    -3
#define TSDBHIP_E_CAPACITY      -4
#define TSDBHIP_E_HIP           -5
#define TSDBHIP_E_RCCL          -6
#define TSDBHIP_E_INVALID_ARG   -7
#define TSDBHIP_E_UNSORTED      -8  /* cells of a span not strictly increasing
                                       after row assembly: input the reference
                                       never produces from compacted rows */
#define TSDBHIP_E_OUT_OF_BOUNDS -9  /* reference would throw
                                       ArrayIndexOutOfBoundsException */
#define TSDBHIP_E_NO_DEVICE    -10
#define TSDBHIP_E_UNSUPPORTED  -11 /* reserved (ABI v2 raised it for a Q1
                                       seek whose shifted reads cross merged
                                       rows; v3 reproduces those reads)      */

/* ---- aggregator op codes (Aggregators.java:44-48 names) --------------- */
#define TSDBHIP_AGG_SUM 0
#define TSDBHIP_AGG_MIN 1
#define TSDBHIP_AGG_MAX 2
#define TSDBHIP_AGG_AVG 3
#define TSDBHIP_AGG_DEV 4

/* tsdbhip_timing.hot_kernel */
#define TSDBHIP_HOT_NONE        0
#define TSDBHIP_HOT_DS_CHUNKS   1 /* k_ds_reg (+ k_ds_spans): streaming decode+downsample */
#define TSDBHIP_HOT_DECODE_FAST 2 /* streaming per-span decode(+downsample) */
#define TSDBHIP_HOT_DECODE_GEN  3 /* general per-span decode(+downsample)   */
#define TSDBHIP_HOT_REDUCE_DIRECT 5 /* k_reduce over direct spans (no-downsampling path) */
#define TSDBHIP_HOT_LOCKSTEP    6 /* k_lockstep: one pass over qualifiers + values of a lockstep group */
#define TSDBHIP_HOT_UG_DS_REG   7 /* k_ug_ds_reg: the uniform aligned group in one launch */
#define TSDBHIP_HOT_UG_DEV      8 /* k_ug_dev: integer dev chains of a uniform group */
#define TSDBHIP_HOT_DS_E        9 /* k_ds_reg in the uniform E variant: the spans' bucket values
                                     on the key's buckets (k_ug_reduce runs after it) */
#define TSDBHIP_HOT_COMPACT     4 /* k_compact_wave: every row's classification and compaction
                                     in one pass (tsdbhip_compact_rows)      */

/* ---- desc flags ------------------------------------------------------- */
#define TSDBHIP_DESC_DEVICE   0x1u /* every array pointer in the desc is a
                                      device pointer (data already in HBM) */
#define TSDBHIP_EXACT_ORDER   0x2u /* reduce over spans strictly in span order
                                      (bit-exact double sums / dev; slower) */
#define TSDBHIP_SHARDED       0x4u /* desc holds this rank's shard of the
                                      group; exchange with the other ranks of
                                      the communicator set by tsdbhip_comm_init */

typedef struct tsdbhip_ctx tsdbhip_ctx;

/*
 * One SpanGroup: the spans (in TreeMap order, TsdbQuery.java:242-243) and
 * the compacted KeyValues of each span, rows sorted by time within a span.
 * qual_bytes / val_bytes hold exactly the KeyValue qualifier()/value() bytes
 * (big-endian, as stored in HBase); a row's qualifier offset must be even.
 */
typedef struct tsdbhip_sg_desc {
  int64_t  start_time;      /* SpanGroup start (u32 held in int64)        */
  int64_t  end_time;        /* SpanGroup end   (u32 held in int64)        */
  uint8_t  rate;            /* SpanGroup.rate                              */
  uint8_t  agg;             /* TSDBHIP_AGG_*  cross-series aggregator      */
  uint8_t  ds_agg;          /* TSDBHIP_AGG_*  downsampler (ds_interval>0)  */
  uint8_t  reserved0;
  uint32_t flags;           /* TSDBHIP_DESC_DEVICE | TSDBHIP_EXACT_ORDER.. */
  int32_t  ds_interval;     /* seconds, 0 = no downsampling                */
  uint32_t n_spans;
  uint64_t n_rows;
  const uint64_t* span_row_start; /* [n_spans+1] rows of span s are
                                     [span_row_start[s], span_row_start[s+1]) */
  const uint32_t* row_base;       /* [n_rows] base_time from the row key      */
  const uint32_t* row_ncells;     /* [n_rows] qualifier().length / 2          */
  const uint64_t* row_qual_off;   /* [n_rows] byte offset into qual_bytes     */
  const uint64_t* row_val_off;    /* [n_rows] byte offset into val_bytes      */
  const uint32_t* row_val_len;    /* [n_rows] value().length                  */
  const uint8_t*  qual_bytes;
  uint64_t        qual_nbytes;
  const uint8_t*  val_bytes;
  uint64_t        val_nbytes;
  uint64_t        span0;    /* TSDBHIP_SHARDED: global index (TreeMap order)
                               of this shard's first span; the ranks agree on
                               the error the reference throws first by global
                               span order (ABI v4). 0 otherwise.           */
} tsdbhip_sg_desc;

/* Result of one SpanGroup, in emission order (SGIterator order). */
typedef struct tsdbhip_sg_out {
  uint64_t capacity;        /* in:  size of ts/is_int/bits                 */
  int64_t* ts;              /* out: DataPoint.timestamp()                  */
  uint8_t* is_int;          /* out: DataPoint.isInteger()                  */
  int64_t* bits;            /* out: longValue() or doubleToRawLongBits()   */
  uint64_t n_out;           /* out: SpanGroup.size()                       */
  uint64_t n_input_points;  /* out: SpanGroup.aggregatedSize()             */
  int32_t  err_code;        /* out: same as the return code                */
  int32_t  reserved0;
  int64_t  err_index;       /* out: first output index not delivered by the
                               lazy reference, or -1 if unknown / no error  */
} tsdbhip_sg_out;

/* Per-call device timings of the last tsdbhip_spangroup_run on a ctx,
 * measured with HIP events on the ctx stream (milliseconds). After
 * tsdbhip_compact_rows: total_ms (the call), and under "timing_detail"
 * hot_ms = k_compact_wave, grid_ms = k_compact_rows, reduce_ms =
 * k_compact_complex + k_compact_dups; hot_kernel = TSDBHIP_HOT_COMPACT. */
typedef struct tsdbhip_timing {
  float    total_ms;        /* first kernel start .. last kernel end        */
  float    decode_ms;       /* decode(+downsample) kernel — dominant, HBM   */
  float    grid_ms;         /* union-grid construction                      */
  float    reduce_ms;       /* cross-span reduction + combine               */
  float    exchange_ms;     /* RCCL exchange (sharded runs, "timing_detail") */
  float    hot_ms;          /* the dominant HBM-streaming kernel alone      */
  uint32_t hot_kernel;      /* TSDBHIP_HOT_*: which kernel hot_ms timed      */
  uint32_t n_collectives;   /* sharded calls: collective launches this rank
                               issued (one per RCCL group)                  */
  uint64_t decode_bytes;    /* algorithmic bytes read+written by decode      */
  uint64_t alg_bytes;       /* SURVEY §8(d) algorithmic bytes of the call   */
  uint64_t n_grid;          /* |G|                                           */
  uint64_t n_emitted;       /* Σ|E_s| (points after downsampling)           */
  uint32_t paths;           /* TSDBHIP_PATH_* bits: which variants ran (ABI v5) */
  uint32_t late_stamp;      /* 1: the call-end stamp (the host's proof that the
                               snapshot and results are this call's) arrived
                               only after the stream sync; summed in totals */
  uint64_t x_bytes;         /* sharded calls: bytes this rank received in the
                               call's collectives (ABI v6)                  */
  uint64_t h2d_bytes;       /* bytes of host-resident inputs the call copied
                               to HBM (a rerun copies none again; ABI v7)  */
} tsdbhip_timing;
/* tsdbhip_timing.paths */
#define TSDBHIP_PATH_ALIGNED_GROUP 1u  /* k_ds_reg's aligned-group reduction
                                          stood for E + the reduce            */
#define TSDBHIP_PATH_ALIGNED_RERUN 2u  /* it was tried, a span fell outside the
                                          group: E rewritten, usual reduce    */
#define TSDBHIP_PATH_LOCKSTEP      4u  /* no downsampling, every span on one
                                          cadence: k_lockstep's single pass   */
#define TSDBHIP_PATH_DIRECT_REDO   8u  /* k_lockstep found a qualifier off the
                                          proposal: the call ran again on the
                                          proven (scan + reduce) path         */
#define TSDBHIP_PATH_UNIFORM      16u  /* every kept span proposed one class key
                                          at assembly: G from the key, no grid
                                          kernels, one host round trip        */
#define TSDBHIP_PATH_UNIFORM_FALLBACK 32u  /* the uniform aligned group did not
                                          stand: the general path ran the call */

/* ---- row compaction (CompactionQueue.compact) -------------------------- */
/*
 * A batch of HBase rows, each a list of KeyValues (qualifier, value) in the
 * order HBase returns them (sorted by qualifier bytes). For every row the
 * library computes compacted[0] of CompactionQueue.compact(row, compacted)
 * (CompactionQueue.java:243-435) — the cell TsdbQuery.findSpans hands to
 * Span.addRow (TsdbQuery.java:264-266).
 *
 * Layout (chosen so the per-KV metadata stays small next to the ~7 bytes of
 * cell data per KV): the qualifiers of row r's KVs are packed back to back,
 * in KV order, in qual_bytes[row_qual_off[r], row_qual_off[r+1]); likewise
 * the values in val_bytes[row_val_off[r], row_val_off[r+1]). Per KV only the
 * two lengths are passed (u16: an OpenTSDB qualifier is at most 2*4096 bytes
 * and a compacted value at most 8*4096+1). Offsets must be non-decreasing
 * and each row's lengths must add up to its extents, else
 * TSDBHIP_E_INVALID_ARG.
 */
typedef struct tsdbhip_rows_desc {
  uint32_t flags;               /* TSDBHIP_DESC_DEVICE: desc AND out arrays
                                   are device pointers                      */
  uint32_t reserved0;
  uint64_t n_rows;
  uint64_t n_kvs;
  const uint64_t* row_kv_start; /* [n_rows+1] KVs of row r                   */
  const uint64_t* row_qual_off; /* [n_rows+1] qualifier bytes of row r       */
  const uint64_t* row_val_off;  /* [n_rows+1] value bytes of row r           */
  const uint16_t* kv_qual_len;  /* [n_kvs] qualifier().length                */
  const uint16_t* kv_val_len;   /* [n_kvs] value().length                    */
  const uint8_t*  qual_bytes;
  uint64_t        qual_nbytes;
  const uint8_t*  val_bytes;
  uint64_t        val_nbytes;
} tsdbhip_rows_desc;

/* Row status codes for tsdbhip_rows_out.row_status */
#define TSDBHIP_ROW_NONE     0  /* compacted[0] stays null (empty / junk)     */
#define TSDBHIP_ROW_SINGLE   1  /* the single KV, possibly float-fixed        */
#define TSDBHIP_ROW_TRIVIAL  2  /* trivialCompact                             */
#define TSDBHIP_ROW_COMPLEX  3  /* complexCompact                             */
#define TSDBHIP_ROW_ERROR    4  /* IllegalDataException                       */
#define TSDBHIP_ROW_OOB      5  /* ArrayIndexOutOfBoundsException
                                   (breakDownValues on a malformed compacted
                                   cell, CompactionQueue.java:708,722)       */

/*
 * Output: row r's compacted qualifier is written at
 *   qual_bytes[row_qual_off[r] - row_qual_off[0]]   (never longer than the
 *   row's input qualifiers), its value at
 *   val_bytes[row_val_off[r] - row_val_off[0] + r]  (never longer than the
 *   row's input values + 1 meta byte),
 * so one pass needs no output scan: qual_capacity >= qualifier extent and
 * val_capacity >= value extent + n_rows. Bytes between rows are undefined.
 * Rows with status NONE/ERROR/OOB have length 0.
 */
typedef struct tsdbhip_rows_out {
  uint64_t qual_capacity;    /* in: bytes available in qual_bytes           */
  uint64_t val_capacity;     /* in: bytes available in val_bytes            */
  uint8_t*  row_status;      /* [n_rows]                                     */
  uint64_t* row_qual_off;    /* [n_rows] offset of the compacted qualifier   */
  uint32_t* row_qual_len;    /* [n_rows]                                     */
  uint64_t* row_val_off;     /* [n_rows]                                     */
  uint32_t* row_val_len;     /* [n_rows]                                     */
  uint8_t*  qual_bytes;      /* out                                          */
  uint8_t*  val_bytes;       /* out                                          */
  uint64_t  qual_used;       /* out: qualifier extent written               */
  uint64_t  val_used;        /* out: value extent written                   */
  uint64_t  n_complex;       /* out: rows that reached complexCompact
                                (status COMPLEX, ERROR or OOB)             */
  /* The write/delete decision of compact() (CompactionQueue.java:276,
   * 355-404, 419-434) for a row whose base time is old enough to be written
   * back (the caller applies the cut-off of :408-413 and
   * TSDB.enable_compactions). Both arrays are optional (NULL: not produced).
   *   row_write[r]   1: tsdb.put(key, compacted qualifier, compacted value)
   *                  (TRIVIAL rows, and COMPLEX rows unless a KV of the row
   *                  already holds exactly the compacted qualifier AND
   *                  value, :388-396); 0 otherwise.
   *   row_keep_kv[r] index, relative to row_kv_start[r], of the KV that
   *                  holds the compacted qualifier (:364-400) and must NOT
   *                  be deleted; -1 if none.
   * The delete set of a TRIVIAL/COMPLEX row (tsdb.delete, :421-434) is every
   * KV of the row whose qualifier length is even and non-zero (junk KVs were
   * dropped from the list, :301-306), except row_keep_kv. SINGLE / NONE /
   * ERROR / OOB rows: no put, no delete (:245-269 return before any write;
   * an exception aborts the row). */
  uint8_t*  row_write;       /* [n_rows] or NULL                             */
  int32_t*  row_keep_kv;     /* [n_rows] or NULL                             */
} tsdbhip_rows_out;

/* ---- synthetic, HBM-resident inputs (bench / tests) -------------------- */
#define TSDBHIP_SYN_INT64_COUNTER 0 /* 8-byte longs (flags 0x7), monotone
                                       counter, increments in (0,1000)       */
#define TSDBHIP_SYN_FLOAT32       1 /* 4-byte floats (flags 0xB), ~100+N(0,1) */
#define TSDBHIP_SYN_FLOAT64       2 /* 8-byte doubles (flags 0xF)             */

typedef struct tsdbhip_synth_params {
  uint64_t seed;
  uint32_t n_spans;
  uint32_t n_points;        /* points per span                              */
  uint32_t t0;              /* first timestamp (divisible by 3600)          */
  uint32_t step;            /* cadence in seconds (divides 3600)            */
  uint32_t kind;            /* TSDBHIP_SYN_*                                */
  uint32_t span0;           /* global index of the first span (shards)      */
} tsdbhip_synth_params;

/* ---- context ----------------------------------------------------------- */
/*
 * A context owns a pool of per-call slots (HIP stream, HBM scratch, pinned
 * staging): every entry point is re-entrant, and calls from several host
 * threads on one context run concurrently, each on its own slot (the
 * reference's Netty workers and gnuplot pool threads call SpanGroup
 * concurrently, GraphHandler.java:182,285). tsdbhip_last_error is the calling
 * thread's last message; tsdbhip_last_timing the calling thread's last call
 * on that context.
 */
int         tsdbhip_open(int32_t device, tsdbhip_ctx** out);
/*
 * One context over several GPUs of this process (the JVM's, TsdbQuery.java:
 * 301-307): tsdbhip_spangroup_run splits each SpanGroup into contiguous span
 * ranges (span order kept, balanced by points for host descs), runs rank r on
 * devices[r] from a host thread of its own, and exchanges grid and partials
 * over RCCL (ncclCommInitAll) when the devices are distinct; when a device
 * repeats, the ranks sharing it exchange through device copies (several
 * shards on one GPU: same results, used to run the N-rank exchange on one
 * GPU). tsdbhip_open_mask: the devices of the set bits of gpu_mask.
 * Compaction, group-by batches, synthetic inputs and probes of a
 * multi-device context run on its first device. */
int         tsdbhip_open_devices(const int32_t* devices, uint32_t n, tsdbhip_ctx** out);
/* Path / diagnostic options of a context and of its member contexts (ABI v6;
 * results never depend on them: the tests use them to run every kernel
 * variant, A/B runs to compare; no environment variable is read):
 *   "decode"        "auto" | "general" | "fast" | "chunks" | "spans" | "direct"
 *   "aligned_group" "on" | "off"   k_ds_reg's aligned-group reduction
 *   "lockstep"      "on" | "off" | "always"   the lockstep proposal (k_lockstep):
 *                   "on" for groups of >= 2048 lockstep waves (and sharded
 *                   groups), "always" for any group
 *   "timing_detail" "on" | "off"   decode / grid event pairs in tsdbhip_timing
 *   "check_clean"   "on" | "off"   check the zero-on-entry invariants (stderr)
 *   "events"        "kernel" | "marker" | "none"   how tsdbhip_timing is measured:
 *                   HIP events carried by the kernel launches (default), event
 *                   markers between kernels (each can idle the GPU a few us),
 *                   or not at all (timings 0)
 * Unknown names or values: TSDBHIP_E_INVALID_ARG. */
int         tsdbhip_set_option(tsdbhip_ctx* ctx, const char* name, const char* value);
int         tsdbhip_open_mask(uint32_t gpu_mask, tsdbhip_ctx** out);
int         tsdbhip_ranks(tsdbhip_ctx* ctx);  /* shards per SpanGroup (1: one device) */
void        tsdbhip_close(tsdbhip_ctx* ctx);
const char* tsdbhip_last_error(tsdbhip_ctx* ctx);
int         tsdbhip_abi_version(void);

int tsdbhip_host_register(tsdbhip_ctx* ctx, void* p, size_t n);
int tsdbhip_host_unregister(tsdbhip_ctx* ctx, void* p);

/* ---- the hot path ------------------------------------------------------ */
int tsdbhip_spangroup_run(tsdbhip_ctx* ctx, const tsdbhip_sg_desc* desc,
                          tsdbhip_sg_out* out);
int tsdbhip_last_timing(tsdbhip_ctx* ctx, tsdbhip_timing* t);
/* Sums of the float timing fields (and of n_grid / n_emitted) over every
 * call on ctx since the last reset, and their count: a caller times many
 * calls without a per-call readout. reset != 0 zeroes them after reading. */
int tsdbhip_timing_totals(tsdbhip_ctx* ctx, tsdbhip_timing* sum, uint64_t* n_calls, int32_t reset);

/* ---- group-by batching ------------------------------------------------- */
/*
 * Every SpanGroup of one query's GROUP BY in one call — the array
 * TsdbQuery.groupByAndAggregate returns (TsdbQuery.java:294-363): the groups
 * share start/end/rate/aggregator/downsampler (one SpanGroup ctor call per
 * group with the query's arguments, TsdbQuery.java:346-348). `desc` holds the
 * spans of all groups, group g's spans being [group_span_start[g],
 * group_span_start[g+1]) in TreeMap order within the group, groups in the
 * ByteMap order of their tag-value keys; group_span_start is a host array of
 * n_groups+1 entries with [0] = 0 and [n_groups] = desc->n_spans. outs[g]
 * receives group g's points exactly as tsdbhip_spangroup_run on that group
 * alone would (same err_code / err_index per group). Returns TSDBHIP_OK, or
 * the first failing group's code (every outs[g].err_code is set). Not with
 * TSDBHIP_SHARDED. Per-call timings: tsdbhip_last_timing.
 */
int tsdbhip_spangroup_run_batch(tsdbhip_ctx* ctx, const tsdbhip_sg_desc* desc, uint32_t n_groups,
                                const uint32_t* group_span_start, tsdbhip_sg_out* outs);

/* ---- output formatting (host cores, no GPU) ----------------------------- */
/*
 * Writes the text the reference's consumers print for n points of one
 * SpanGroup (tsdbhip_sg_out arrays) into buf:
 *   TSDBHIP_FMT_ASCII   "<metric> <ts> <value><tags>\n"   GraphHandler.respondAsciiQuery
 *                        (GraphHandler.java:785-808); tags = " k=v k2=v2" as the
 *                        caller built it from getTags()
 *   TSDBHIP_FMT_GNUPLOT "<ts + utc_offset> <value>\n"     Plot.dumpToFiles (Plot.java:190-204)
 *   TSDBHIP_FMT_CLI     "<metric> <ts> <value> <tags>\n"  CliQuery (CliQuery.java:161-170);
 *                        tags = getTags().toString(), doubles as String.format("%f")
 * Longs as Long.toString, doubles as Double.toString (JDK 19+ shortest
 * digits). Returns the bytes written, TSDBHIP_E_CAPACITY if cap is too small
 * (nothing written), TSDBHIP_E_NAN_INF for a NaN/Infinity in ASCII/GNUPLOT
 * (the reference's IllegalStateException), TSDBHIP_E_INVALID_ARG.
 */
#define TSDBHIP_FMT_ASCII   0
#define TSDBHIP_FMT_GNUPLOT 1
#define TSDBHIP_FMT_CLI     2
int64_t tsdbhip_format_points(int32_t mode, const char* metric, const char* tags, int64_t utc_offset,
                              const int64_t* ts, const uint8_t* is_int, const int64_t* bits, uint64_t n,
                              char* buf, uint64_t cap);

/* ---- secondary path ---------------------------------------------------- */
int tsdbhip_compact_rows(tsdbhip_ctx* ctx, const tsdbhip_rows_desc* desc,
                         tsdbhip_rows_out* out);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI -------------------- */
#define TSDBHIP_UNIQUE_ID_BYTES 128
int tsdbhip_comm_unique_id(uint8_t out[TSDBHIP_UNIQUE_ID_BYTES]);
int tsdbhip_comm_init(tsdbhip_ctx* ctx, int32_t nranks, int32_t rank,
                      const uint8_t id[TSDBHIP_UNIQUE_ID_BYTES]);

/* ---- device-resident synthetic SpanGroup ------------------------------- */
/* Generates the KeyValue bytes of a synthetic SpanGroup directly in HBM
 * (same bytes as opentsdb_amd.synth on the host) and fills *desc with device
 * pointers owned by ctx (flags |= TSDBHIP_DESC_DEVICE). Free with
 * tsdbhip_synth_free. Only n_spans/n_points/... of params are used; the
 * query fields of *desc (start/end/agg/...) are left for the caller. */
int tsdbhip_synth_generate(tsdbhip_ctx* ctx, const tsdbhip_synth_params* p,
                           tsdbhip_sg_desc* desc);
int tsdbhip_synth_free(tsdbhip_ctx* ctx, tsdbhip_sg_desc* desc);

/* Copies the device-resident desc's arrays back to host buffers sized by the
 * desc (for parity checks of the generator). */
int tsdbhip_desc_download(tsdbhip_ctx* ctx, const tsdbhip_sg_desc* ddesc,
                          uint64_t* span_row_start, uint32_t* row_base,
                          uint32_t* row_ncells, uint64_t* row_qual_off,
                          uint64_t* row_val_off, uint32_t* row_val_len,
                          uint8_t* qual_bytes, uint8_t* val_bytes);

/* ---- measurement ------------------------------------------------------- */
/* Bandwidth probe over a device-resident desc (TSDBHIP_DESC_DEVICE):
 * mode 0 streams its qualifier + value rows with the geometry of the
 * downsampling kernel (one wave per span, 16-B loads), mode 1 copies its
 * value bytes device-to-device, mode 2 is a flat grid-stride read of the
 * value bytes, mode 3 is mode 0 with two chunks in flight per wave and the
 * next span's metadata loaded ahead (width 8, single-row spans).
 * *ms = kernel time, *bytes = bytes moved.
 * `width` = value bytes per cell (4 or 8). Not part of the reference API:
 * it reports the achievable bandwidth beside the 8 TB/s peak. */
int tsdbhip_bw_probe(tsdbhip_ctx* ctx, const tsdbhip_sg_desc* desc, int32_t mode, uint32_t width,
                     float* ms, uint64_t* bytes);

#ifdef __cplusplus
}
#endif
#endif /* TSDBHIP_H */
