// k_decode.hip — RowSeq cell decode + Span.DownsamplingIterator, one wave per
// kept span, producing the span's emitted sequence E_s (SURVEY.md §8a,
// "closed-form restatement"):
//   * cells are decoded exactly as RowSeq.Iterator does (RowSeq.java:385-455):
//     ts = base + (q >>> 4), value at the running offset (incl. quirk Q1 and
//     the `short` value_index overflow), RowSeq.extract*Value (:194-226);
//   * E_s starts at the first cell >= start (Span.Iterator.seek, Span.java:280-287);
//   * with downsampling, buckets are greedy (Span.java:377-422): a bucket
//     starts at the first unconsumed point p and holds every point with
//     ts < p.ts + interval; its ts is floor(sum ts / n); integer iff all its
//     points are; the value is ds.runLong / ds.runDouble(toDouble) over the
//     bucket (Span.java:476-511), evaluated in point order.
//
// Layout in HBM: E arrays are SoA, span k's points at [e_off[k], e_off[k] +
// e_len[k]): e_ts u32, e_val i64 (long or raw double bits), e_flt u8.
//
// Per 64-cell chunk: lanes decode one cell each; bucket starts are found by a
// ballot chain; integer-path sums/min/max (associative, exact) come from wave
// scans. Order-dependent double sums and Welford (dev) are evaluated by one
// lane per bucket in point order (exact). A span runs in FAST mode (integer
// path only) until it meets a float cell, then restarts in SEQ mode.
#pragma once
#include "dev_common.h"

namespace tsdb {

struct DecodeArgs {
  const uint64_t* span_row_start;
  const uint32_t* row_base;
  const uint64_t* row_qual_off;
  const uint64_t* row_val_off;
  const uint8_t* qual;
  const uint8_t* val;
  const uint8_t* row_ok;
  const uint32_t* row_cell0;
  const uint32_t* kept;       // [n_kept] span index of kept span k
  uint32_t n_kept;
  const uint32_t* sp_ncells;
  const int64_t* sp_q1;
  const int32_t* sp_q1_shift;
  const int64_t* sp_q1_rs;    // [2 n_spans] the seek RowSeq's rows [rs0, rs1)
  const uint32_t* row_ncells;
  const uint32_t* row_val_len;
  const int64_t* sp_ovf_cell;
  const uint64_t* sp_cap;
  const uint64_t* e_off;      // [n_kept]
  uint32_t* e_ts;
  int64_t* e_val;
  uint8_t* e_flt;
  uint32_t* e_len;            // [n_kept]
  int64_t* e_bad;             // [n_kept] (first bad E index << 4) | code id, or -1
  int64_t start, end;
  int32_t interval;           // 0 = no downsampling
  int32_t ds_agg;
  int32_t rate;
  unsigned long long* err;  // [1] first error (err_raise key)
  uint64_t span0;           // global index of span 0 (error order across shards)
  unsigned int* gflags;       // [0] any float E point, [1] any int E point
  unsigned long long* range;  // [0] min grid-candidate ts, [1] max E ts
  unsigned long long* fstar;  // max first-E ts over spans whose first E point is float
  uint32_t* fb_list;          // spans the fast kernel handed to the general one
  uint32_t* fb_count;         // [1]; general kernels iterate this list when `use_fb`
  int32_t use_fb;
  const uint32_t* span_list;  // k_decode_fast: spans to take (null = all kept)
  const uint32_t* span_count;
  const int64_t* sp_first;    // [n_spans] first accepted ts (k_decode_rows)
};

#define BAD_ILLEGAL 1
#define BAD_OOB 2

struct CellChunk {
  bool valid, in_e, isflt, okv;
  int64_t ts;
  int64_t bits;
};

// Quirk Q1 across merged rows (RowSeq.java:405-421): the RowSeq's values
// array is its rows' value bytes (meta bytes stripped) concatenated
// (RowSeq.java:152-165); a cell at offset `off` of its row `row` is read at
// its merged offset minus `shift`, gathered byte by byte from the rows
// [rs0, rs1) (the read may start in an earlier row or straddle two).
DEVI uint32_t dec_row_vbytes(const DecodeArgs& a, uint64_t q) {
  const uint32_t n = a.row_ncells[q], vl = a.row_val_len[q];
  return n > 1 && vl > 0 ? vl - 1 : vl;
}
DEVI bool q1_merged_read(const DecodeArgs& a, uint64_t rs0, uint64_t rs1, uint64_t row, uint64_t off, int32_t shift,
                         uint32_t fl, int64_t* bits) {
  uint64_t acc = 0;
  for (uint64_t q = rs0; q < row; q++)
    if (a.row_ok[q]) acc += dec_row_vbytes(a, q);
  const uint64_t p = acc + off - (uint64_t)(int64_t)shift;
  const uint32_t lm = fl & 7;
  const uint32_t len = (fl & 8) ? (lm == 7 ? 8u : 4u) : lm + 1;
  uint64_t u = 0, seg = 0, q = rs0;
  for (uint32_t b = 0; b < len; b++) {
    const uint64_t pos = p + b;
    while (q < rs1 && (!a.row_ok[q] || pos >= seg + dec_row_vbytes(a, q))) {
      if (a.row_ok[q]) seg += dec_row_vbytes(a, q);
      q++;
    }
    const uint32_t byte = q < rs1 ? a.val[a.row_val_off[q] + (pos - seg)] : 0u;
    u = (u << 8) | byte;
  }
  return decode_be(u, fl, bits);
}

// Decodes cell c0+lane of span (rows [r0,r1)). Carries the running value
// offset of the row that continues into the next chunk.
DEVI void decode_chunk(const DecodeArgs& a, uint64_t r0, uint64_t r1, uint32_t n, uint32_t c0,
                       int64_t q1_row, int32_t q1_shift, int64_t ovf_cell,
                       int64_t& carry_row, uint64_t& carry_off, CellChunk& o, uint64_t q1_rs0 = 0,
                       uint64_t q1_rs1 = 0) {
  const int lane = lane_id();
  const uint32_t c = c0 + lane;
  o.valid = c < n;
  int64_t row = -1;
  uint32_t len = 0, fl = 0;
  if (o.valid) {
    // last row with row_cell0 <= c (dropped rows share the next row's prefix)
    uint64_t lo = r0, hi = r1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (a.row_cell0[mid] <= c) lo = mid + 1; else hi = mid;
    }
    row = (int64_t)lo - 1;
    const uint32_t ci = c - a.row_cell0[row];
    const uint32_t q = load_qual(a.qual, a.row_qual_off[row] + 2ull * ci);
    o.ts = (int64_t)a.row_base[row] + (q >> 4);
    fl = q & 15;
    len = (fl & 7) + 1;
  } else {
    o.ts = INT64_MAX;
  }
  // running value offset within the row: segmented scan of the lengths
  const int64_t prow = (int64_t)shfl_up_u64((uint64_t)row, 1);
  const bool head = lane == 0 || prow != row;
  const uint64_t hmask = ballot(head);
  const uint32_t incl = wave_seg_scan_u32(len, hmask);
  uint64_t off = incl - len;
  const uint64_t first_seg = (hmask & ~1ull) ? lanemask_lt(__builtin_ctzll(hmask & ~1ull)) : ~0ull;
  if (((first_seg >> lane) & 1) && row == carry_row) off += carry_off;
  // carry for the next chunk: the row of the last valid lane
  const int lastv = (int)((n - c0) < 64u ? (n - c0) : 64u) - 1;
  const int64_t lrow = (int64_t)readlane_u64((uint64_t)row, lastv);
  const uint64_t loff = readlane_u64(off + len, lastv);
  carry_row = lrow;
  carry_off = loff;
  o.in_e = o.valid && o.ts >= a.start;
  o.isflt = (fl & 8) != 0;
  o.okv = true;
  o.bits = 0;
  if (o.valid) {
    const bool q1 = q1_row >= 0 && o.in_e && row >= q1_row && (uint64_t)row < q1_rs1;  // quirk Q1
    if (q1 && (q1_rs0 != (uint64_t)q1_row || q1_rs1 != (uint64_t)q1_row + 1))
      o.okv = q1_merged_read(a, q1_rs0, q1_rs1, (uint64_t)row, off, q1_shift, fl, &o.bits);
    else if (o.in_e)  // (a one-row RowSeq: its own bytes, shifted)
      o.okv = decode_value(a.val, a.row_val_off[row] + off - (q1 ? (uint64_t)(int64_t)q1_shift : 0ull), fl, &o.bits);
    if ((int64_t)c >= ovf_cell && ovf_cell >= 0) o.okv = false;
  }
}

__device__ void span_nods_general(const DecodeArgs& a, uint32_t k);

__global__ void __launch_bounds__(256) k_decode_nods(DecodeArgs a) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t n = a.use_fb ? *a.fb_count : a.n_kept;
  for (uint32_t i = wave; i < n; i += nwaves) span_nods_general(a, a.use_fb ? a.fb_list[i] : i);
}

__device__ void span_nods_general(const DecodeArgs& a, uint32_t k) {
  const int lane = lane_id();
  {
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    const uint32_t n = a.sp_ncells[s];
    const int64_t q1_row = a.sp_q1[s], ovf = a.sp_ovf_cell[s];
    const int32_t q1_shift = a.sp_q1_shift[s];
    const uint64_t q1_rs0 = q1_row >= 0 ? (uint64_t)a.sp_q1_rs[2ull * s] : 0ull;
    const uint64_t q1_rs1 = q1_row >= 0 ? (uint64_t)a.sp_q1_rs[2ull * s + 1] : 0ull;
    const uint64_t eo = a.e_off[k];
    int64_t carry_row = -1; uint64_t carry_off = 0;
    int64_t prev_ts = -1;
    uint32_t nskip = 0;
    int64_t bad = -1;
    bool unsorted = false, anyf = false, anyi = false;
    for (uint32_t c0 = 0; c0 < n; c0 += WAVE) {
      CellChunk o;
      decode_chunk(a, r0, r1, n, c0, q1_row, q1_shift, ovf, carry_row, carry_off, o, q1_rs0, q1_rs1);
      int64_t pts = (int64_t)shfl_up_u64((uint64_t)o.ts, 1);
      if (lane == 0) pts = prev_ts;
      if (ballot(o.valid && o.ts <= pts) != 0) unsorted = true;
      prev_ts = (int64_t)readlane_u64((uint64_t)o.ts, (int)((n - c0) < 64u ? (n - c0) : 64u) - 1);
      nskip += __popcll(ballot(o.valid && !o.in_e));
      const uint32_t e = c0 + lane - nskip;
      if (o.in_e) {
        a.e_ts[eo + e] = (uint32_t)o.ts;
        a.e_val[eo + e] = o.bits;
        a.e_flt[eo + e] = o.isflt;
      }
      const uint64_t bm = ballot(o.in_e && !o.okv);
      if (bad < 0 && bm) {
        const int bl = __builtin_ctzll(bm);
        const uint32_t be = readlane_u32(e, bl);
        const int64_t code = ((int64_t)(c0 + bl) >= ovf && ovf >= 0) ? BAD_OOB : BAD_ILLEGAL;
        bad = ((int64_t)be << 4) | code;
      }
      anyf |= ballot(o.in_e && o.isflt) != 0;
      anyi |= ballot(o.in_e && !o.isflt) != 0;
    }
    const uint32_t len = n - nskip;
    if (lane == 0) {
      a.e_len[k] = len;
      a.e_bad[k] = bad;
      if (unsorted) err_raise(a.err, 2, a.span0 + s, -8 /*E_UNSORTED*/);
      if (anyf) atomicOr(&a.gflags[0], 1u);
      if (anyi) atomicOr(&a.gflags[1], 1u);
    }
  }
}

// Block (256 threads) per kept span, no downsampling: spans of many short
// rows (C4: ~11k one-cell hourly rows a span) decoded row-parallel, a thread
// per row, instead of the wave walk whose every 64 cells each binary-search
// their row (k_decode_nods). Taken when the span's E is its accepted cells
// in order (first point >= start, no Q1 seek, no `short` overflow): cell c
// of the span (row_cell0 prefix) is E[c]. Otherwise wave 0 runs the general
// walk. RowSeq.java:360-497 (ts = base + delta, values at the running
// offset of the row), :194-226 (widths); unsorted cells: E_UNSORTED, as the
// walk raises it.
#ifndef DR_THREADS
#define DR_THREADS 512  // threads a span (C4 step: 256 9.98 ms, 512 9.93, 1024 9.96)
#endif
__global__ void __launch_bounds__(DR_THREADS) k_decode_rows(DecodeArgs a) {
  constexpr uint32_t NW = DR_THREADS / WAVE;
  __shared__ unsigned long long s_bad[NW];
  __shared__ uint32_t s_f[NW], s_i[NW], s_uns[NW];
  const uint32_t k = blockIdx.x;
  if (k >= a.n_kept) return;
  const uint32_t s = a.kept[k];
  const bool rowpar = a.sp_q1[s] < 0 && a.sp_ovf_cell[s] < 0 && a.sp_first[s] >= a.start;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (!rowpar) {
    if (w == 0) span_nods_general(a, k);
    return;
  }
  const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
  const uint64_t eo = a.e_off[k];
  unsigned long long bad = ~0ull;
  bool anyf = false, anyi = false, uns = false;
  for (uint64_t r = r0 + t; r < r1; r += DR_THREADS) {
    if (!a.row_ok[r]) continue;
    const uint32_t n = a.row_ncells[r], c0 = a.row_cell0[r];
    const uint64_t qo = a.row_qual_off[r], vo = a.row_val_off[r];
    const int64_t base = a.row_base[r];
    uint64_t off = 0;
    int64_t prev = -1;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t q = load_qual(a.qual, qo + 2ull * i);
      const uint32_t fl = q & 15;
      const int64_t ts = base + (q >> 4);
      int64_t bits = 0;
      const bool ok = decode_value(a.val, vo + off, fl, &bits);
      off += (fl & 7) + 1;
      const uint64_t e = (uint64_t)c0 + i;
      a.e_ts[eo + e] = (uint32_t)ts;
      a.e_val[eo + e] = bits;
      a.e_flt[eo + e] = (fl & 8) ? 1 : 0;
      if (!ok) bad = min(bad, (unsigned long long)((e << 4) | BAD_ILLEGAL));
      if (fl & 8) anyf = true; else anyi = true;
      if (i && ts <= prev) uns = true;
      prev = ts;
    }
  }
  __syncthreads();  // (every E point of the span written by this block)
  __threadfence_block();
  // a row's first cell against the cell before it (the previous accepted row's last)
  for (uint64_t r = r0 + t; r < r1; r += DR_THREADS) {
    if (!a.row_ok[r] || a.row_ncells[r] == 0) continue;
    const uint32_t c0 = a.row_cell0[r];
    if (c0 > 0 && a.e_ts[eo + c0] <= a.e_ts[eo + c0 - 1]) uns = true;
  }
  for (int o = 1; o < WAVE; o <<= 1) bad = min(bad, (unsigned long long)shfl_xor_u64(bad, o));
  const uint64_t fm = ballot(anyf), im = ballot(anyi), um = ballot(uns);
  if (lane == 0) {
    s_bad[w] = bad;
    s_f[w] = fm != 0;
    s_i[w] = im != 0;
    s_uns[w] = um != 0;
  }
  __syncthreads();
  if (t == 0) {
    unsigned long long b = ~0ull;
    uint32_t fu = 0, ff = 0, fi = 0;
    for (uint32_t i = 0; i < NW; i++) {
      b = min(b, s_bad[i]);
      fu |= s_uns[i];
      ff |= s_f[i];
      fi |= s_i[i];
    }
    a.e_len[k] = a.sp_ncells[s];
    a.e_bad[k] = b == ~0ull ? -1 : (int64_t)b;
    if (fu) err_raise(a.err, 2, a.span0 + s, -8 /*E_UNSORTED*/);
    if (ff) atomicOr(&a.gflags[0], 1u);
    if (fi) atomicOr(&a.gflags[1], 1u);
  }
}

// ------------------------------------------------------------ downsample ---
struct Bucket {
  int64_t end;      // first ts + interval
  uint32_t n;
  uint32_t nflt;
  uint64_t tssum;
  int64_t ia;       // int path: sum / min / max
  double dsum;      // double path
  double dmm;       // double min / max
  Welford wf;       // dev
  bool bad;
};

template <int AGG>
DEVI int64_t ia_combine(int64_t x, int64_t y) {  // x earlier, y later
  if (AGG == 1) return y < x ? y : x;            // min: keep first of equals
  if (AGG == 2) return y > x ? y : x;            // max
  return ladd(x, y);                              // sum / avg
}

template <int AGG>
DEVI void seq_push(Bucket& b, double x, bool first) {
  if (first) { b.dsum = x; b.dmm = x; }
  else {
    b.dsum += x;
    if (AGG == 1) { if (x < b.dmm) b.dmm = x; }
    if (AGG == 2) { if (x > b.dmm) b.dmm = x; }
  }
  if (AGG == 4) wf_push(b.wf, x);
}

template <int AGG>
DEVI void finalize_bucket(const DecodeArgs& a, const Bucket& b, uint64_t eidx, uint64_t eo) {
  const uint64_t ts = b.tssum / b.n;  // Span.java:399 newtime /= npoints
  const bool allint = b.nflt == 0;
  int64_t v;
  if (allint) {
    if (AGG == 3) v = ldiv(b.ia, (int64_t)b.n);
    else if (AGG == 4) v = d2l(wf_result(b.wf));
    else v = b.ia;
  } else {
    double d;
    if (AGG == 0) d = b.dsum;
    else if (AGG == 3) d = b.dsum / (double)(int32_t)b.n;
    else if (AGG == 4) d = wf_result(b.wf);
    else d = b.dmm;
    v = dbits(d);
  }
  a.e_ts[eo + eidx] = (uint32_t)ts;
  a.e_val[eo + eidx] = v;
  a.e_flt[eo + eidx] = !allint;
}

// One span, any row structure (general path; also the fallback of the fast
// kernel). s_bits/s_flt: this wave's 64-entry LDS staging.
template <int AGG>
__device__ void span_ds_general(const DecodeArgs& a, uint32_t k, int64_t* s_bits_w, uint8_t* s_flt_w) {
  const int lane = lane_id();
  {
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    const uint32_t n = a.sp_ncells[s];
    const int64_t q1_row = a.sp_q1[s], ovf = a.sp_ovf_cell[s];
    const int32_t q1_shift = a.sp_q1_shift[s];
    const uint64_t q1_rs0 = q1_row >= 0 ? (uint64_t)a.sp_q1_rs[2ull * s] : 0ull;
    const uint64_t q1_rs1 = q1_row >= 0 ? (uint64_t)a.sp_q1_rs[2ull * s + 1] : 0ull;
    const uint64_t eo = a.e_off[k], cap = a.sp_cap[s];
    // dev always needs the ordered Welford; others start FAST (int path only)
    bool seq = (AGG == 4);
  restart:
    int64_t carry_row = -1; uint64_t carry_off = 0;
    int64_t prev_ts = -1;
    bool unsorted = false, anyf = false, anyi = false;
    int64_t bad = -1;
    uint64_t ecount = 0;
    bool open = false;
    Bucket cb;  // carried open bucket (wave-uniform)
    cb.end = 0; cb.n = 0; cb.nflt = 0; cb.tssum = 0; cb.ia = 0; cb.dsum = 0; cb.dmm = 0;
    wf_init(cb.wf); cb.bad = false;
    for (uint32_t c0 = 0; c0 < n; c0 += WAVE) {
      CellChunk o;
      decode_chunk(a, r0, r1, n, c0, q1_row, q1_shift, ovf, carry_row, carry_off, o, q1_rs0, q1_rs1);
      const int lastv = (int)((n - c0) < 64u ? (n - c0) : 64u) - 1;
      int64_t pts = (int64_t)shfl_up_u64((uint64_t)o.ts, 1);
      if (lane == 0) pts = prev_ts;
      if (ballot(o.valid && o.ts <= pts) != 0) unsorted = true;
      prev_ts = (int64_t)readlane_u64((uint64_t)o.ts, lastv);
      const uint64_t emask = ballot(o.in_e);
      if (!emask) continue;
      const uint64_t fmask = ballot(o.in_e && o.isflt);
      if (fmask && !seq) { seq = true; goto restart; }
      anyf |= fmask != 0;
      anyi |= (emask & ~fmask) != 0;
      const uint64_t badmask = ballot(o.in_e && !o.okv);
      // ---- greedy bucket chain (Span.java:389-398) ----
      uint64_t starts = 0;
      int64_t E = open ? cb.end : INT64_MIN;
      uint64_t cand = emask;
      for (;;) {
        const uint64_t m = ballot(o.in_e && o.ts >= E) & cand;
        if (!m) break;
        const int l = __builtin_ctzll(m);
        starts |= 1ull << l;
        E = (int64_t)readlane_u64((uint64_t)o.ts, l) + a.interval;
        cand &= ~lanemask_le(l);
      }
      const int fe = __builtin_ctzll(emask);
      const int le = 63 - __builtin_clzll(emask);
      const bool cont = open && !((starts >> fe) & 1);
      if (open && !cont) {
        // the carried bucket ended exactly at the chunk boundary: emit it
        if (lane == 0 && ecount < cap) finalize_bucket<AGG>(a, cb, ecount, eo);
        if (bad < 0 && cb.bad) bad = ((int64_t)ecount << 4) | BAD_ILLEGAL;
        ecount++;
        open = false;
      }
      const uint64_t heads = starts | (cont ? (1ull << fe) : 0ull);
      const int nseg = __popcll(heads);
      // this lane's segment bounds (lane j describes segment j)
      int seg_a = 64, seg_b = -1;
      if (lane < nseg) {
        seg_a = select_bit(heads, lane);
        const uint64_t ab = heads & ~lanemask_le(seg_a);
        seg_b = ab ? __builtin_ctzll(ab) - 1 : le;
      }
      // ---- integer-path scans ----
      const uint64_t tsv = o.in_e ? (uint64_t)o.ts : 0;
      const uint64_t S_ts = wave_incl_scan_u64(tsv);
      int64_t S_ia;
      if (AGG == 0 || AGG == 3) {
        S_ia = (int64_t)wave_incl_scan_u64(o.in_e ? (uint64_t)o.bits : 0);
      } else if (AGG == 1 || AGG == 2) {
        // segmented inclusive min/max scan over heads
        int64_t x = o.bits;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int64_t y = (int64_t)shfl_up_u64((uint64_t)x, d);
          const uint64_t win = (lane >= d) ? (lanemask_le(lane) & ~lanemask_le(lane - d)) : 0;
          if (lane >= d && (heads & win) == 0) x = ia_combine<AGG>(y, x);
        }
        S_ia = x;
      } else {
        S_ia = 0;
      }
      // gather per-segment totals onto lane j
      const int ga = seg_a < 64 ? seg_a : 0, gb = seg_b >= 0 ? seg_b : 0;
      const uint64_t ts_b = shfl_u64(S_ts, gb);
      const uint64_t ts_a = shfl_u64(S_ts, ga > 0 ? ga - 1 : 0);
      const int64_t ia_b = (int64_t)shfl_u64((uint64_t)S_ia, gb);
      const int64_t ia_a = (int64_t)shfl_u64((uint64_t)S_ia, ga > 0 ? ga - 1 : 0);
      Bucket b;
      if (lane < nseg) {
        const uint64_t rm = lanemask_le(seg_b) & ~lanemask_lt(seg_a);
        b.n = (uint32_t)(seg_b - seg_a + 1);
        b.nflt = (uint32_t)__popcll(fmask & rm);
        b.tssum = ts_b - (seg_a > 0 ? ts_a : 0);
        if (AGG == 0 || AGG == 3) b.ia = (int64_t)((uint64_t)ia_b - (seg_a > 0 ? (uint64_t)ia_a : 0));
        else b.ia = ia_b;
        b.bad = (badmask & rm) != 0;
        b.end = 0;
        b.dsum = 0; b.dmm = 0; wf_init(b.wf);
      }
      // ---- ordered double path / Welford: one lane per segment ----
      if (seq) {
        s_bits_w[lane] = o.bits;
        s_flt_w[lane] = o.isflt;
        wave_lds_sync();
        if (lane < nseg) {
          bool first = true;
          if (lane == 0 && cont) { b.dsum = cb.dsum; b.dmm = cb.dmm; b.wf = cb.wf; first = false; }
          for (int i = seg_a; i <= seg_b; i++) {
            const double x = to_double(s_bits_w[i], s_flt_w[i] != 0);
            seq_push<AGG>(b, x, first);
            first = false;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      // continuation merges the carried integer-path state
      if (lane == 0 && cont && nseg > 0) {
        b.n += cb.n; b.nflt += cb.nflt; b.tssum += cb.tssum;
        b.ia = ia_combine<AGG>(cb.ia, b.ia);
        b.bad = b.bad || cb.bad;
      }
      // ---- close buckets: every segment but the last, and the last one at span end ----
      const bool span_end = c0 + WAVE >= n;
      const int nclosed = span_end ? nseg : nseg - 1;
      if (lane < nclosed) {
        const uint64_t eidx = ecount + lane;
        if (eidx < cap) finalize_bucket<AGG>(a, b, eidx, eo);
      }
      const uint64_t bl = ballot(lane < nclosed && b.bad);
      if (bad < 0 && bl) bad = ((int64_t)(ecount + __builtin_ctzll(bl)) << 4) | BAD_ILLEGAL;
      ecount += nclosed;
      // carry the last (open) segment
      if (!span_end && nseg > 0) {
        const int j = nseg - 1;
        cb.n = readlane_u32(b.n, j);
        cb.nflt = readlane_u32(b.nflt, j);
        cb.tssum = readlane_u64(b.tssum, j);
        cb.ia = (int64_t)readlane_u64((uint64_t)b.ia, j);
        cb.bad = readlane_u32(b.bad ? 1u : 0u, j) != 0;
        cb.dsum = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.dsum), j));
        cb.dmm = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.dmm), j));
        cb.wf.n = (int64_t)readlane_u64((uint64_t)b.wf.n, j);
        cb.wf.mean = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.wf.mean), j));
        cb.wf.var = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.wf.var), j));
        cb.end = E;
        open = true;
      } else {
        open = false;
      }
    }
    if (lane == 0) {
      a.e_len[k] = (uint32_t)(ecount < cap ? ecount : cap);
      if (ecount > cap) err_raise(a.err, 2, a.span0 + s, -4 /*E_CAPACITY*/);
      a.e_bad[k] = bad;
      if (unsorted) err_raise(a.err, 2, a.span0 + s, -8 /*E_UNSORTED*/);
      if (anyf) atomicOr(&a.gflags[0], 1u);
      if (anyi) atomicOr(&a.gflags[1], 1u);
    }
  }
}

template <int AGG>
__global__ void __launch_bounds__(256) k_decode_ds(DecodeArgs a) {
  __shared__ int64_t s_bits[4][WAVE];
  __shared__ uint8_t s_flt[4][WAVE];
  const int wib = threadIdx.x / WAVE;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t n = a.use_fb ? *a.fb_count : a.n_kept;
  for (uint32_t i = wave; i < n; i += nwaves)
    span_ds_general<AGG>(a, a.use_fb ? a.fb_list[i] : i, s_bits[wib], s_flt[wib]);
}

// Per-span summary of E after decode: empty spans (E_EMPTY_SPAN) and F*
// (the latest first point that is a float). Over `list` only when given: the
// spans k_ds_spans finished are integer and non-empty. Grid-stride, one
// atomic per block and field.
__global__ void __launch_bounds__(256) k_span_summary(DecodeArgs a, const uint32_t* list, const uint32_t* count) {
  __shared__ int64_t sh_fs[4], sh_e[4];
  int64_t fs = 0, empty = 0;
  const uint32_t n = list ? *count : a.n_kept;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = list ? list[i] : i;
    const uint32_t len = a.e_len[k];
    const uint64_t eo = a.e_off[k];
    if (len == 0) {
      empty = 1;
      continue;
    }
    if (!a.rate && a.e_flt[eo]) fs = max(fs, (int64_t)a.e_ts[eo] + 1);  // +1: 0 = none
  }
  auto mx = [](int64_t x, int64_t y) { return max(x, y); };
  fs = block_reduce_256(fs, mx, sh_fs);
  empty = block_reduce_256(empty, mx, sh_e);
  if (threadIdx.x == 0) {
    if (empty) err_raise(a.err, 2, 0, -3 /*E_EMPTY_SPAN*/);
    if (fs) atomicMax(a.fstar, (unsigned long long)fs);
  }
}

}  // namespace tsdb
