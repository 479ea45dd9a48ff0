/*
 * abi_check.c — a C consumer of include/tsdbhip.h, the way the JNI shim of
 * INTEGRATION.md binds it (the consumer of DataPoints.java:23-142 and
 * CompactionQueue.compact, CompactionQueue.java:243-435).
 *
 *   abi_check layout   prints sizeof / offsetof of every struct the header
 *                      declares as JSON (tests/test_abi.py compares them
 *                      with opentsdb_amd/_abi.py's ctypes mirror), then
 *                      formats two points through tsdbhip_format_points
 *                      (host code, no GPU)
 *   abi_check run      on device 0: one SpanGroup (known answer KA-1 of
 *                      SURVEY.md §8(c), int lerp + sum, SpanGroup.java:
 *                      702-730) and one trivially compacted row
 *                      (CompactionQueue.java:450-474), checked against the
 *                      expected values; exit status 0 = pass
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "tsdbhip.h"

#define F(st, f) printf("%s\"%s\": [%zu, %zu]", first++ ? ", " : "", #f, offsetof(st, f), sizeof(((st*)0)->f))
#define BEGIN(st) do { int first = 0; printf("%s\"%s\": {\"size\": %zu, \"fields\": {", nst++ ? ", " : "", #st, sizeof(st))
#define END() printf("}}"); } while (0)

static int layout(void) {
  int nst = 0;
  printf("{\"abi_version\": %d, \"structs\": {", TSDBHIP_ABI_VERSION);
  BEGIN(tsdbhip_sg_desc);
  F(tsdbhip_sg_desc, start_time); F(tsdbhip_sg_desc, end_time); F(tsdbhip_sg_desc, rate);
  F(tsdbhip_sg_desc, agg); F(tsdbhip_sg_desc, ds_agg); F(tsdbhip_sg_desc, reserved0);
  F(tsdbhip_sg_desc, flags); F(tsdbhip_sg_desc, ds_interval); F(tsdbhip_sg_desc, n_spans);
  F(tsdbhip_sg_desc, n_rows); F(tsdbhip_sg_desc, span_row_start); F(tsdbhip_sg_desc, row_base);
  F(tsdbhip_sg_desc, row_ncells); F(tsdbhip_sg_desc, row_qual_off); F(tsdbhip_sg_desc, row_val_off);
  F(tsdbhip_sg_desc, row_val_len); F(tsdbhip_sg_desc, qual_bytes); F(tsdbhip_sg_desc, qual_nbytes);
  F(tsdbhip_sg_desc, val_bytes); F(tsdbhip_sg_desc, val_nbytes); F(tsdbhip_sg_desc, span0);
  END();
  BEGIN(tsdbhip_sg_out);
  F(tsdbhip_sg_out, capacity); F(tsdbhip_sg_out, ts); F(tsdbhip_sg_out, is_int); F(tsdbhip_sg_out, bits);
  F(tsdbhip_sg_out, n_out); F(tsdbhip_sg_out, n_input_points); F(tsdbhip_sg_out, err_code);
  F(tsdbhip_sg_out, reserved0); F(tsdbhip_sg_out, err_index);
  END();
  BEGIN(tsdbhip_timing);
  F(tsdbhip_timing, total_ms); F(tsdbhip_timing, decode_ms); F(tsdbhip_timing, grid_ms);
  F(tsdbhip_timing, reduce_ms); F(tsdbhip_timing, exchange_ms); F(tsdbhip_timing, hot_ms);
  F(tsdbhip_timing, hot_kernel); F(tsdbhip_timing, n_collectives); F(tsdbhip_timing, decode_bytes);
  F(tsdbhip_timing, alg_bytes); F(tsdbhip_timing, n_grid); F(tsdbhip_timing, n_emitted);
  F(tsdbhip_timing, paths); F(tsdbhip_timing, late_stamp); F(tsdbhip_timing, x_bytes); F(tsdbhip_timing, h2d_bytes);
  END();
  BEGIN(tsdbhip_rows_desc);
  F(tsdbhip_rows_desc, flags); F(tsdbhip_rows_desc, reserved0); F(tsdbhip_rows_desc, n_rows);
  F(tsdbhip_rows_desc, n_kvs); F(tsdbhip_rows_desc, row_kv_start); F(tsdbhip_rows_desc, row_qual_off);
  F(tsdbhip_rows_desc, row_val_off); F(tsdbhip_rows_desc, kv_qual_len); F(tsdbhip_rows_desc, kv_val_len);
  F(tsdbhip_rows_desc, qual_bytes); F(tsdbhip_rows_desc, qual_nbytes); F(tsdbhip_rows_desc, val_bytes);
  F(tsdbhip_rows_desc, val_nbytes);
  END();
  BEGIN(tsdbhip_rows_out);
  F(tsdbhip_rows_out, qual_capacity); F(tsdbhip_rows_out, val_capacity); F(tsdbhip_rows_out, row_status);
  F(tsdbhip_rows_out, row_qual_off); F(tsdbhip_rows_out, row_qual_len); F(tsdbhip_rows_out, row_val_off);
  F(tsdbhip_rows_out, row_val_len); F(tsdbhip_rows_out, qual_bytes); F(tsdbhip_rows_out, val_bytes);
  F(tsdbhip_rows_out, qual_used); F(tsdbhip_rows_out, val_used); F(tsdbhip_rows_out, n_complex);
  F(tsdbhip_rows_out, row_write); F(tsdbhip_rows_out, row_keep_kv);
  END();
  BEGIN(tsdbhip_synth_params);
  F(tsdbhip_synth_params, seed); F(tsdbhip_synth_params, n_spans); F(tsdbhip_synth_params, n_points);
  F(tsdbhip_synth_params, t0); F(tsdbhip_synth_params, step); F(tsdbhip_synth_params, kind);
  F(tsdbhip_synth_params, span0);
  END();
  printf("}");
  /* the formatter from C (GraphHandler.respondAsciiQuery's line) */
  const int64_t ts[2] = {1356998400, 1356998410};
  const uint8_t isi[2] = {1, 0};
  int64_t bits[2] = {42, 0};
  const double half = 0.5;
  memcpy(&bits[1], &half, 8);
  char buf[256];
  const int64_t n = tsdbhip_format_points(TSDBHIP_FMT_ASCII, "sys.cpu", " host=a", 0, ts, isi, bits, 2, buf, sizeof buf);
  printf(", \"format\": \"");
  for (int64_t i = 0; i < n; i++) printf(buf[i] == '\n' ? "\\n" : "%c", buf[i]);
  printf("\"}\n");
  return n > 0 ? 0 : 1;
}

static void be64(uint8_t* p, int64_t v) {
  for (int b = 0; b < 8; b++) p[b] = (uint8_t)((uint64_t)v >> (56 - 8 * b));
}

#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
                                       fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); return 1; } } while (0)

static int run(void) {
  tsdbhip_ctx* ctx = NULL;
  int rc = tsdbhip_open(0, &ctx);
  CHECK(rc == TSDBHIP_OK, "tsdbhip_open: %d (%s)", rc, tsdbhip_last_error(NULL));

  /* KA-1: span A {T+100: 10, T+110: 20}, span B {T+105: 100, T+115: 200},
   * 8-byte longs (flags 0x7), one compacted hourly row each (values + the
   * 0x00 meta byte). SpanGroup sum: T+100 -> 10, T+105 -> 15 + 100 (A's lerp
   * truncates), T+110 -> 20 + 150, T+115 -> 200. */
  const int64_t T = 1356998400;
  const uint32_t d[4] = {100, 110, 105, 115};
  const int64_t v[4] = {10, 20, 100, 200};
  uint8_t qual[8], val[34];
  for (int i = 0; i < 4; i++) {
    const uint16_t q = (uint16_t)((d[i] << 4) | 0x7);
    qual[2 * i] = (uint8_t)(q >> 8);
    qual[2 * i + 1] = (uint8_t)q;
    be64(val + 17 * (i / 2) + 8 * (i % 2), v[i]);
  }
  val[16] = val[33] = 0;
  const uint64_t srs[3] = {0, 1, 2};
  const uint32_t base[2] = {(uint32_t)T, (uint32_t)T}, ncells[2] = {2, 2}, vlen[2] = {17, 17};
  const uint64_t qoff[2] = {0, 4}, voff[2] = {0, 17};
  tsdbhip_sg_desc g;
  memset(&g, 0, sizeof g);
  g.start_time = 0;
  g.end_time = 0xFFFFFFFFll;
  g.agg = TSDBHIP_AGG_SUM;
  g.n_spans = 2;
  g.n_rows = 2;
  g.span_row_start = srs; g.row_base = base; g.row_ncells = ncells; g.row_qual_off = qoff;
  g.row_val_off = voff; g.row_val_len = vlen;
  g.qual_bytes = qual; g.qual_nbytes = sizeof qual; g.val_bytes = val; g.val_nbytes = sizeof val;
  int64_t ots[8], obits[8];
  uint8_t oisi[8];
  tsdbhip_sg_out o;
  memset(&o, 0, sizeof o);
  o.capacity = 8; o.ts = ots; o.is_int = oisi; o.bits = obits;
  rc = tsdbhip_spangroup_run(ctx, &g, &o);
  CHECK(rc == TSDBHIP_OK, "tsdbhip_spangroup_run: %d (%s)", rc, tsdbhip_last_error(ctx));
  const int64_t ets[4] = {T + 100, T + 105, T + 110, T + 115}, ev[4] = {10, 115, 170, 200};
  CHECK(o.n_out == 4 && o.n_input_points == 4 && o.err_code == 0, "n_out %llu n_in %llu",
        (unsigned long long)o.n_out, (unsigned long long)o.n_input_points);
  for (int i = 0; i < 4; i++)
    CHECK(ots[i] == ets[i] && oisi[i] == 1 && obits[i] == ev[i], "point %d: %lld %d %lld", i,
          (long long)ots[i], oisi[i], (long long)obits[i]);

  /* one row of two single-cell KVs (deltas 0 and 1 s, 8-byte longs):
   * trivialCompact concatenates the qualifiers and values and appends 0 */
  uint8_t cq[4] = {0x00, 0x07, 0x00, 0x17}, cv[16];
  be64(cv, 7);
  be64(cv + 8, 9);
  const uint64_t kvs[2] = {0, 2}, rq[2] = {0, 4}, rv[2] = {0, 16};
  const uint16_t kql[2] = {2, 2}, kvl[2] = {8, 8};
  tsdbhip_rows_desc rd;
  memset(&rd, 0, sizeof rd);
  rd.n_rows = 1; rd.n_kvs = 2; rd.row_kv_start = kvs; rd.row_qual_off = rq; rd.row_val_off = rv;
  rd.kv_qual_len = kql; rd.kv_val_len = kvl; rd.qual_bytes = cq; rd.qual_nbytes = 4;
  rd.val_bytes = cv; rd.val_nbytes = 16;
  uint8_t st = 0xFF, wr = 0xFF, oq[64], ov[64];
  uint64_t oqo = 9, ovo = 9;
  uint32_t oql = 0, ovl = 0;
  int32_t keep = 7;
  tsdbhip_rows_out ro;
  memset(&ro, 0, sizeof ro);
  ro.qual_capacity = sizeof oq; ro.val_capacity = sizeof ov; ro.row_status = &st; ro.row_qual_off = &oqo;
  ro.row_qual_len = &oql; ro.row_val_off = &ovo; ro.row_val_len = &ovl; ro.qual_bytes = oq; ro.val_bytes = ov;
  ro.row_write = &wr; ro.row_keep_kv = &keep;
  rc = tsdbhip_compact_rows(ctx, &rd, &ro);
  CHECK(rc == TSDBHIP_OK, "tsdbhip_compact_rows: %d (%s)", rc, tsdbhip_last_error(ctx));
  CHECK(st == TSDBHIP_ROW_TRIVIAL && oql == 4 && ovl == 17 && wr == 1 && keep == -1 && ro.n_complex == 0,
        "status %d qlen %u vlen %u write %d keep %d", st, oql, ovl, wr, keep);
  CHECK(memcmp(oq + oqo, cq, 4) == 0, "compacted qualifier");
  CHECK(memcmp(ov + ovo, cv, 16) == 0 && ov[ovo + 16] == 0, "compacted value");

  tsdbhip_timing tm;
  CHECK(tsdbhip_last_timing(ctx, &tm) == TSDBHIP_OK, "tsdbhip_last_timing");
  tsdbhip_close(ctx);
  printf("abi_check run: KA-1 SpanGroup and a trivial compaction bit-exact through the C-ABI\n");
  return 0;
}

int main(int argc, char** argv) {
  if (tsdbhip_abi_version() != TSDBHIP_ABI_VERSION) {
    fprintf(stderr, "library ABI %d, header ABI %d\n", tsdbhip_abi_version(), TSDBHIP_ABI_VERSION);
    return 2;
  }
  if (argc > 1 && !strcmp(argv[1], "run")) return run();
  return layout();
}
