// k_assemble.hip — span assembly: which compacted rows a Span keeps and how
// they group into RowSeqs, per Span.addRow (Span.java:87-132) and
// RowSeq.addRow (RowSeq.java:92-172); the SpanGroup keep rule S7
// (SpanGroup.java:130-142); per-span E capacities.
//
// One wave per span. The common case (rows in strictly increasing base order,
// each row starting after the previous one ended, no RowSeq merge possible)
// is verified wave-parallel; anything else falls back to an exact sequential
// walk by lane 0 (the reference's own algorithm, O(rows)).
#pragma once
#include "dev_common.h"

namespace tsdb {


struct AssembleArgs {
  // input desc (device)
  const uint64_t* span_row_start;
  const uint32_t* row_base;
  const uint32_t* row_ncells;
  const uint64_t* row_qual_off;
  const uint32_t* row_val_len;
  const uint8_t* qual;
  uint32_t n_spans;
  int64_t start, end;
  int32_t interval;  // 0 = no downsampling
  // outputs
  uint8_t* row_ok;        // [n_rows] 0 dropped, 1 merged into the previous
                          // RowSeq, 2 starts a RowSeq
  uint32_t* row_cell0;    // [n_rows] accepted-cell prefix within the span
  uint32_t* sp_ncells;    // [n_spans] Span.size()
  int64_t* sp_first;      // [n_spans] Span.timestamp(0)
  int64_t* sp_last;       // [n_spans] Span.timestamp(size-1)
  uint8_t* sp_kept;       // [n_spans] S7
  uint64_t* sp_cap;       // [n_spans] E capacity (0 if not kept)
  int64_t* sp_q1;         // [n_spans] Q1: row read with shifted offsets, -1 none
  int32_t* sp_q1_shift;   // [n_spans]
  int64_t* sp_q1_rs;      // [2 n_spans] rows [rs0, rs1) of the RowSeq the seek lands in
  int64_t* sp_ovf_cell;   // [n_spans] span cell index that overflows the
                          // RowSeq.Iterator `short` value_index, -1 none
  unsigned long long* err;  // [1] first error (err_raise key)
  uint64_t span0;           // global index of span 0 (a shard's offset): the
                            // error order across ranks is the global span order
  // the uniform-group proposal (spangroup_run's uniform path; null: not
  // made): per span its class key (x0 << 32 | n, step << 32 | q0), ~0 in the
  // first word when the span proposes none, and its row's byte offsets
  const uint64_t* row_val_off;
  uint64_t* u_key1;
  uint64_t* u_key2;
  uint64_t* u_vo;
  uint64_t* u_qo;
};

DEVI int64_t row_first_ts(const AssembleArgs& a, uint64_t r) {
  return (int64_t)a.row_base[r] + (load_qual(a.qual, a.row_qual_off[r]) >> 4);
}
DEVI int64_t row_last_ts(const AssembleArgs& a, uint64_t r) {
  const uint32_t n = a.row_ncells[r];
  return (int64_t)a.row_base[r] + (load_qual(a.qual, a.row_qual_off[r] + 2ull * (n - 1)) >> 4);
}
DEVI uint32_t row_value_bytes(const AssembleArgs& a, uint64_t r) {
  // value bytes without the compacted meta byte (CompactionQueue.java:469-470)
  const uint32_t n = a.row_ncells[r], vl = a.row_val_len[r];
  return n > 1 && vl > 0 ? vl - 1 : vl;
}


// Exact sequential Span.addRow emulation for one span (lane 0 only).
__device__ void assemble_slow(const AssembleArgs& a, uint32_t s, uint64_t r0, uint64_t r1) {
  int64_t rs_base = -1;       // base of the current (last) RowSeq
  uint64_t rs_start = 0;      // first accepted row of the current RowSeq
  uint32_t rs_vbytes = 0;     // value bytes in the current RowSeq
  int64_t last_ts = 0;        // last cell ts of the last RowSeq
  int64_t ovf_cell = -1;
  for (uint64_t r = r0; r < r1; r++) a.row_ok[r] = 0;
  for (uint64_t r = r0; r < r1; r++) {
    const uint32_t n = a.row_ncells[r];
    if (n == 0) { err_raise(a.err, 0, err_scan_order(a.row_base[r], a.span0 + s), -9 /*E_OUT_OF_BOUNDS*/); return; }
    const int64_t base = a.row_base[r];
    const int64_t first = row_first_ts(a, r), last = row_last_ts(a, r);
    if (rs_base < 0) {
      a.row_ok[r] = 2; rs_base = base; rs_start = r; rs_vbytes = row_value_bytes(a, r); last_ts = last;
      continue;
    }
    if (last - rs_base < 4096) {  // merge into the last RowSeq (Span.java:117-121)
      const int64_t time_adj = base - rs_base;
      if (time_adj <= 0) {
        if (time_adj != 0) { err_raise(a.err, 0, err_scan_order((uint32_t)base, a.span0 + s), -1 /*E_ILLEGAL_DATA*/); return; }
        // same row again (scanner restart): RowSeq restarts from this row
        for (uint64_t q = rs_start; q < r; q++) a.row_ok[q] = 0;
        a.row_ok[r] = 2; rs_start = r; rs_vbytes = row_value_bytes(a, r); last_ts = last;
        continue;
      }
      if (last_ts >= first) continue;  // RowSeq.java:142-148: row ignored
      a.row_ok[r] = 1;
      rs_vbytes += row_value_bytes(a, r);
      last_ts = last;
      continue;
    }
    if (last_ts >= first) continue;  // Span.java:126-130: RowSeq dropped
    a.row_ok[r] = 2; rs_base = base; rs_start = r; rs_vbytes = row_value_bytes(a, r); last_ts = last;
  }
  (void)rs_vbytes;
  // prefix of accepted cells; RowSeq grouping for the `short` overflow and Q1
  uint32_t c = 0;
  rs_base = -1;
  uint32_t cum = 0;           // value bytes so far in the current RowSeq
  uint32_t rs_cell0 = 0;
  int64_t first_ts = -1, last_all = 0;
  uint64_t first_row = r1, seek_rs_row0 = r1, seek_rs_cell0 = 0;
  bool seek_found = false;
  uint64_t last_rs_row0 = r1; uint32_t last_rs_cell0 = 0;
  for (uint64_t r = r0; r < r1; r++) {
    a.row_cell0[r] = c;
    if (!a.row_ok[r]) continue;
    const uint32_t n = a.row_ncells[r];
    const int64_t base = a.row_base[r];
    const int64_t last = row_last_ts(a, r);
    if (first_row == r1) { first_row = r; first_ts = row_first_ts(a, r); }
    if (a.row_ok[r] == 2) {  // starts a new RowSeq (recorded by the walk above)
      rs_base = base; cum = 0; rs_cell0 = c;
      last_rs_row0 = r; last_rs_cell0 = c;
    }
    // overflow of RowSeq.Iterator.value_index (a Java short)
    if (ovf_cell < 0 && cum + row_value_bytes(a, r) >= 32768u) {
      uint32_t run = cum;
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t q = load_qual(a.qual, a.row_qual_off[r] + 2ull * i);
        run += (q & 7) + 1;
        if (run >= 32768u) { ovf_cell = (int64_t)c + i; break; }
      }
    }
    cum += row_value_bytes(a, r);
    if (!seek_found && last >= a.start) {  // seekRow: first RowSeq with last ts >= start
      seek_found = true; seek_rs_row0 = last_rs_row0; seek_rs_cell0 = last_rs_cell0;
    }
    (void)rs_cell0;
    last_all = last;
    c += n;
  }
  a.sp_ncells[s] = c;
  a.sp_first[s] = first_ts;
  a.sp_last[s] = last_all;
  a.sp_ovf_cell[s] = ovf_cell;
  a.sp_q1[s] = -1;
  a.sp_q1_shift[s] = 0;
  // Q1 (RowSeq.java:405-421): seek skips cells with the stale qualifier.
  if (c > 0 && first_ts < a.start && seek_found) {
    uint32_t k = 0, slen = 0;
    uint64_t rows_in_rs = 0, crow = r1;
    bool done = false;
    for (uint64_t r = seek_rs_row0; r < r1 && !done; r++) {
      if (!a.row_ok[r]) continue;
      if (r != seek_rs_row0 && a.row_ok[r] == 2) break;
      rows_in_rs++;
      const uint32_t n = a.row_ncells[r];
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t q = load_qual(a.qual, a.row_qual_off[r] + 2ull * i);
        if ((int64_t)a.row_base[r] + (q >> 4) >= a.start) { crow = r; done = true; break; }
        k++; slen += (q & 7) + 1;
      }
    }
    const int32_t shift = (int32_t)slen - (int32_t)k;
    // the seek RowSeq ends at the next row that starts a RowSeq: its cells from
    // the seek on are read at their offsets in the merged values array minus
    // the shift, across its merged rows (RowSeq.java:92-172, 405-421)
    uint64_t rs1 = r1;
    for (uint64_t r = crow + 1; r < r1; r++)
      if (a.row_ok[r] == 2) { rs1 = r; break; }
    if (shift != 0) {
      a.sp_q1[s] = (int64_t)crow;
      a.sp_q1_shift[s] = shift;
      a.sp_q1_rs[2ull * s] = (int64_t)seek_rs_row0;
      a.sp_q1_rs[2ull * s + 1] = (int64_t)rs1;
    }
    (void)seek_rs_cell0;
    (void)rows_in_rs;
  }
}

// S7 keep rule and the span's E capacity (lane 0 / the span's thread).
DEVI void assemble_finish(const AssembleArgs& a, uint32_t s, bool has_rows) {
  const uint32_t n = a.sp_ncells[s];
  const int64_t f = a.sp_first[s], l = a.sp_last[s];
  // Span.timestamp(0) of an empty span throws (SpanGroup.java:135-139)
  (void)has_rows;
  if (n == 0) err_raise(a.err, 1, a.span0 + s, -3 /*E_EMPTY_SPAN*/);
  const bool kept = n > 0 && f <= a.end && l >= a.start;  // SpanGroup.java:135-139
  a.sp_kept[s] = kept;
  uint64_t cap = 0;
  if (kept) {
    cap = n;
    if (a.interval > 0) {
      const int64_t lo = f > a.start ? f : a.start;
      const uint64_t b = (uint64_t)((l - lo) / a.interval) + 1;
      cap = b < cap ? b : cap;
    }
  }
  a.sp_cap[s] = cap;
}

// One thread per span: the common case (at most ASM_ROWS rows, each starting
// after the previous one ended with no RowSeq merge possible, no seek inside
// the first row) written directly; every other span is queued for the
// wave-per-span kernel below. (A thread walks its rows one dependent load
// chain after the other: spans of many rows — a day of hourly rows — go to
// the wave kernel, which loads 64 rows at once.)
constexpr uint32_t ASM_ROWS = 4;
// The uniform-group proposal of a span of n >= 2 cells whose rows all passed
// the assembly checks (one RowSeq a row, no Q1 / overflow): one value width
// W (8 or 4 B) in its first row, the qualifiers of the first row's cells 0
// and 1 and of the last row's last cell on ts = x0 + c*step with one flags
// nibble, every point inside [start, end]. Spans proposing one key are one
// cadence each (RowSeq.java:360-497), so their union grid is that cadence
// (SpanGroup.java:510-608), downsampled: one bucket sequence; the kernels
// that take the group prove every other qualifier as they stream (k_lockstep,
// k_ds_reg). Bit 16 of k2: a span of several rows (k_lockstep and k_ug_dev
// read one row a span; k_ds_reg any).
DEVI bool ug_probe(const AssembleArgs& a, uint64_t r0, uint64_t r1, uint32_t n, uint64_t& k1, uint64_t& k2,
                   uint64_t& vo, uint64_t& qo) {
  const bool one = r1 - r0 == 1;
  const uint32_t n0 = one ? n : a.row_ncells[r0];
  if (n0 < 2) return false;
  const uint32_t vb = a.row_val_len[r0] - 1;  // (n0 >= 2: a compacted row ends with its meta byte)
  const uint32_t W = vb / n0;
  qo = a.row_qual_off[r0];
  vo = a.row_val_off[r0];
  if (!((W == 8 || W == 4) && vb == W * n0 && (qo & 1) == 0 && (vo & (W - 1)) == 0)) return false;
  const uint64_t rl = r1 - 1;
  const uint32_t nl = one ? n : a.row_ncells[rl];
  const uint64_t qol = one ? qo : a.row_qual_off[rl];
  const uint32_t q0 = load_qual(a.qual, qo), q1 = load_qual(a.qual, qo + 2), ql = load_qual(a.qual, qol + 2ull * (nl - 1));
  const uint32_t fl = q0 & 15u;
  const uint32_t d0 = q0 >> 4, d1 = q1 >> 4, dl = ql >> 4;
  if (!((fl & 7u) == W - 1 && (q1 & 15u) == fl && (ql & 15u) == fl && d1 > d0)) return false;
  const uint32_t step = d1 - d0;
  const int64_t first = (int64_t)a.row_base[r0] + d0;
  const int64_t last = first + (int64_t)(n - 1) * step;
  if ((int64_t)a.row_base[rl] + dl != last) return false;
  if (!(first >= a.start && last <= a.end && last < (1ll << 32))) return false;
  k1 = ((uint64_t)first << 32) | n;
  k2 = ((uint64_t)step << 32) | (one ? 0u : 0x10000u) | q0;
  return true;
}

// The thread-per-span case for span s (< n_spans); true: deferred to the
// wave walk.
DEVI bool assemble_fast_one(const AssembleArgs& a, uint32_t s) {
  bool defer = false;
  {
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    bool ok = r1 > r0 && r1 - r0 <= ASM_ROWS;
    int64_t pb = -1, pl = -1, first_ts = 0;
    uint32_t cell = 0;
    for (uint64_t r = r0; ok && r < r1; r++) {
      const uint32_t n = a.row_ncells[r];
      if (n == 0 || row_value_bytes(a, r) >= 32768u) { ok = false; break; }
      const int64_t base = a.row_base[r], first = row_first_ts(a, r), last = row_last_ts(a, r);
      if (pb >= 0 && (base <= pb || first <= pl || last - pb < 4096)) { ok = false; break; }
      if (r == r0) {
        if (first < a.start) { ok = false; break; }  // Q1 seek inside the row
        first_ts = first;
      }
      pb = base;
      pl = last;
      cell += n;
    }
    if (ok) {
      uint32_t c = 0;
      for (uint64_t r = r0; r < r1; r++) {  // (second pass: rows written only after the checks)
        a.row_ok[r] = 2;
        a.row_cell0[r] = c;
        c += a.row_ncells[r];
      }
      a.sp_ncells[s] = cell;
      a.sp_first[s] = first_ts;
      a.sp_last[s] = pl;
      a.sp_ovf_cell[s] = -1;
      a.sp_q1[s] = -1;
      a.sp_q1_shift[s] = 0;
      assemble_finish(a, s, true);
    } else {
      defer = true;
    }
    if (a.u_key1) {  // (a deferred span proposes nothing)
      uint64_t k1 = ~0ull, k2 = 0, vo = 0, qo = 0;
      if (ok && cell >= 2 && !ug_probe(a, r0, r1, cell, k1, k2, vo, qo)) k1 = ~0ull;
      a.u_key1[s] = k1;
      a.u_key2[s] = k2;
      a.u_vo[s] = vo;
      a.u_qo[s] = qo;
    }
  }
  return defer;
}

__global__ void __launch_bounds__(256) k_assemble_fast(AssembleArgs a, uint32_t* list, uint32_t* count) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const bool defer = s < a.n_spans && assemble_fast_one(a, s);
  // queue the deferred spans (one atomic per wave)
  const uint64_t m = ballot(defer);
  if (m) {
    uint32_t base = 0;
    if (lane_id() == __ffsll((long long)m) - 1) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (defer) list[base + __popcll(m & lanemask_lt(lane_id()))] = s;
  }
}

// Span.addRow / RowSeq.addRow walk (the first loop of assemble_slow) with
// the rows' metadata loaded 64 at a time by the wave and the decision chain
// run uniformly over lanes (readlane): exact for every span whose rows never
// restart a RowSeq (time_adj <= 0), never overflow the `short` value index,
// and whose first accepted cell is at or after start (no seek inside a row).
// Returns false (nothing written that the slow walk does not rewrite) when
// the span needs the slow walk.
DEVI bool assemble_walk(const AssembleArgs& a, uint32_t s, uint64_t r0, uint64_t r1) {
  const int lane = lane_id();
  int64_t rs_base = -1, last_ts = 0;
  uint32_t cum = 0;           // value bytes of the current RowSeq
  uint32_t cell = 0;
  int64_t first_ts = -1, last_all = 0;
  for (uint64_t rb = r0; rb < r1; rb += WAVE) {
    const uint64_t r = rb + lane;
    const bool valid = r < r1;
    uint32_t n = 0, base = 0, fdt = 0, ldt = 0, vb = 0;
    if (valid) {
      n = a.row_ncells[r];
      base = a.row_base[r];
      if (n > 0) {
        fdt = load_qual(a.qual, a.row_qual_off[r]) >> 4;
        ldt = load_qual(a.qual, a.row_qual_off[r] + 2ull * (n - 1)) >> 4;
        vb = row_value_bytes(a, r);
      }
    }
    if (ballot(valid && n == 0)) return false;  // (the slow walk reports it)
    const uint32_t nb = (uint32_t)min((uint64_t)WAVE, r1 - rb);
    uint32_t st = 0;  // this lane's row: 0 dropped, 1 merged, 2 starts a RowSeq
    for (uint32_t j = 0; j < nb; j++) {
      const int64_t b = (int64_t)readlane_u32(base, (int)j);
      const int64_t first = b + readlane_u32(fdt, (int)j), last = b + readlane_u32(ldt, (int)j);
      const uint32_t v = readlane_u32(vb, (int)j);
      uint32_t x = 0;
      if (rs_base < 0) {
        x = 2; rs_base = b; last_ts = last; cum = v;
      } else if (last - rs_base < 4096) {  // merge into the last RowSeq (Span.java:117-121)
        if (b - rs_base <= 0) return false;  // restart / illegal: slow walk
        if (last_ts < first) { x = 1; last_ts = last; cum += v; }  // else RowSeq.java:142-148
      } else if (last_ts < first) {        // else Span.java:126-130: dropped
        x = 2; rs_base = b; last_ts = last; cum = v;
      }
      if (cum >= 32768u) return false;     // short value_index overflow: slow walk
      if (x && first_ts < 0) first_ts = first;
      if (x) last_all = last;
      st = lane == (int)j ? x : st;
    }
    const uint32_t acc = st ? n : 0u;
    const uint32_t incl = wave_incl_scan_u32(acc);
    if (valid) {
      a.row_ok[r] = (uint8_t)st;
      a.row_cell0[r] = cell + incl - acc;
    }
    cell += readlane_u32(incl, 63);
  }
  if (first_ts < a.start) return false;  // seek inside the first RowSeq (Q1): slow walk
  if (lane == 0) {
    a.sp_ncells[s] = cell;
    a.sp_first[s] = first_ts;
    a.sp_last[s] = last_all;
    a.sp_ovf_cell[s] = -1;
    a.sp_q1[s] = -1;
    a.sp_q1_shift[s] = 0;
  }
  return true;
}

// The walk above for spans whose rows come in strictly increasing base and
// time order and where no RowSeq can take a third row (last(r) - base(r-2)
// >= 4096, e.g. hourly rows with seconds of jitter past the hour). Span.java:117
// then reduces to merge(r) = c(r) && !merge(r-1), with c(r) = last(r) -
// base(r-1) < 4096: a row merges into a RowSeq its predecessor started.
// Along a run of rows with c set, merges alternate from the run's first row,
// so the decisions of 64 rows come from one ballot instead of a 64-step
// readlane chain (the chain is issue-bound: C4, a day of jittered hourly
// rows per span, spent 3.5 ms in it). Returns false, with nothing written
// that the next walk does not rewrite, when a precondition fails.
DEVI bool assemble_walk_pairs(const AssembleArgs& a, uint32_t s, uint64_t r0, uint64_t r1) {
  const int lane = lane_id();
  int64_t pb1 = -1, pl1 = -1, pb2 = -1;  // base/last of row r-1, base of row r-2 (previous batch)
  uint32_t pv1 = 0;                      // value bytes of row r-1
  bool pm1 = false;                      // row r-1 merged
  uint32_t cell = 0;
  int64_t first_ts = -1, last_all = 0;
  // the next batch's row fields are loaded while this batch's qualifiers are
  // (the walk is a chain of batches, two dependent loads each otherwise)
  uint32_t n_n = 0, vl_n = 0;
  int64_t base_n = 0;
  uint64_t qo_n = 0;
  auto load_rows = [&](uint64_t rb) {
    const uint64_t r = rb + lane;
    n_n = vl_n = 0;
    base_n = 0;
    qo_n = 0;
    if (r < r1) {
      n_n = a.row_ncells[r];
      vl_n = a.row_val_len[r];
      base_n = a.row_base[r];
      qo_n = a.row_qual_off[r];
    }
  };
  load_rows(r0);
  for (uint64_t rb = r0; rb < r1; rb += WAVE) {
    const uint64_t r = rb + lane;
    const bool valid = r < r1;
    const uint32_t n = n_n;
    const int64_t base = base_n;
    const uint64_t qo = qo_n;
    // (row_value_bytes: without the compacted meta byte, CompactionQueue.java:469-470)
    const uint32_t vb = valid && n > 0 ? (n > 1 && vl_n > 0 ? vl_n - 1 : vl_n) : 0u;
    int64_t first = 0, last = 0;
    if (valid && n > 0) {
      first = base + (load_qual(a.qual, qo) >> 4);
      last = base + (load_qual(a.qual, qo + 2ull * (n - 1)) >> 4);
    }
    if (rb + WAVE < r1) load_rows(rb + WAVE);
    if (ballot(valid && n == 0)) return false;
    const uint32_t nb = (uint32_t)min((uint64_t)WAVE, r1 - rb);
    int64_t b1 = (int64_t)shfl_up_u64((uint64_t)base, 1);
    int64_t l1 = (int64_t)shfl_up_u64((uint64_t)last, 1);
    uint32_t v1 = shfl_up_u32(vb, 1);
    int64_t b2 = (int64_t)shfl_up_u64((uint64_t)base, 2);
    if (lane == 0) { b1 = pb1; l1 = pl1; v1 = pv1; b2 = pb2; }
    if (lane == 1) b2 = pb1;
    const bool has1 = r > r0, has2 = r > r0 + 1;
    const bool bad = valid && ((has1 && (base <= b1 || first <= l1)) || (has2 && last - b2 < 4096));
    if (ballot(bad)) return false;
    const bool c = valid && has1 && last - b1 < 4096;
    const uint64_t cm = ballot(c);
    const uint64_t zero = ~cm & lanemask_le(lane);  // rows up to this one that cannot merge
    bool m;
    if (zero) {
      const int h = 63 - __clzll((long long)zero);
      m = c && ((lane - h - 1) & 1) == 0;
    } else {
      m = c && ((lane & 1) == (pm1 ? 1 : 0));  // run continues from the previous batch
    }
    // the RowSeq's value bytes must stay below the short index (else the slow walk)
    if (ballot(valid && (m ? v1 + vb : vb) >= 32768u)) return false;
    const uint32_t incl = wave_incl_scan_u32(n);
    if (valid) {
      a.row_ok[r] = (uint8_t)(m ? 1 : 2);
      a.row_cell0[r] = cell + incl - n;
    }
    cell += readlane_u32(incl, 63);
    if (rb == r0) first_ts = (int64_t)readlane_u64((uint64_t)first, 0);
    const int t = (int)nb - 1;
    pb2 = nb >= 2 ? (int64_t)readlane_u64((uint64_t)base, t - 1) : pb1;
    pb1 = (int64_t)readlane_u64((uint64_t)base, t);
    pl1 = (int64_t)readlane_u64((uint64_t)last, t);
    pv1 = readlane_u32(vb, t);
    pm1 = (ballot(m) >> t) & 1;
    last_all = pl1;
  }
  if (first_ts < a.start) return false;  // seek inside the first RowSeq (Q1): slow walk
  if (lane == 0) {
    a.sp_ncells[s] = cell;
    a.sp_first[s] = first_ts;
    a.sp_last[s] = last_all;
    a.sp_ovf_cell[s] = -1;
    a.sp_q1[s] = -1;
    a.sp_q1_shift[s] = 0;
  }
  return true;
}

// One wave per span (of `list`, or of all spans when list is null). The
// common case (rows in strictly increasing base order, each row starting
// after the previous one ended, no RowSeq merge possible) is verified
// wave-parallel; anything else falls back to an exact sequential walk by
// lane 0 (the reference's own algorithm, O(rows)).
DEVI void assemble_span_wave(const AssembleArgs& a, uint32_t s) {
  const int lane = lane_id();
  {
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    bool ok = r1 > r0;
    int64_t prev_last = -1, prev_base = -1;
    uint32_t cell = 0;
    bool q1 = false;
    for (uint64_t rb = r0; rb < r1 && ok; rb += WAVE) {
      const uint64_t r = rb + lane;
      const bool valid = r < r1;
      uint32_t n = valid ? a.row_ncells[r] : 0;
      int64_t base = 0, first = 0, last = 0;
      if (valid && n > 0) { base = a.row_base[r]; first = row_first_ts(a, r); last = row_last_ts(a, r); }
      int64_t pb = (int64_t)shfl_up_u64((uint64_t)base, 1);
      int64_t pl = (int64_t)shfl_up_u64((uint64_t)last, 1);
      if (lane == 0) { pb = prev_base; pl = prev_last; }
      bool bad = valid && (n == 0 || row_value_bytes(a, r) >= 32768u ||
                           (pb >= 0 && (base <= pb || first <= pl || last - pb < 4096)));
      if (valid && r == r0 && first < a.start) q1 = true;
      if (ballot(bad) != 0 || ballot(q1) != 0) { ok = false; break; }
      const uint32_t incl = wave_incl_scan_u32(n);
      if (valid) { a.row_ok[r] = 2; a.row_cell0[r] = cell + incl - n; }
      cell += readlane_u32(incl, 63);
      prev_base = (int64_t)readlane_u64((uint64_t)base, 63);
      prev_last = (int64_t)readlane_u64((uint64_t)last, 63);
      const uint64_t nv = r1 - rb;
      if (nv < WAVE) {
        prev_base = (int64_t)readlane_u64((uint64_t)base, (int)nv - 1);
        prev_last = (int64_t)readlane_u64((uint64_t)last, (int)nv - 1);
      }
    }
    if (ok) {
      if (lane == 0) {
        a.sp_ncells[s] = cell;
        a.sp_first[s] = row_first_ts(a, r0);
        a.sp_last[s] = prev_last;
        a.sp_ovf_cell[s] = -1;
        a.sp_q1[s] = -1;
        a.sp_q1_shift[s] = 0;
        if (a.u_key1) {  // (a span of many rows: the proposal here, not in k_assemble_fast)
          uint64_t k1 = ~0ull, k2 = 0, vo = 0, qo = 0;
          if (cell >= 2 && !ug_probe(a, r0, r1, cell, k1, k2, vo, qo)) k1 = ~0ull;
          a.u_key1[s] = k1;
          a.u_key2[s] = k2;
          a.u_vo[s] = vo;
          a.u_qo[s] = qo;
        }
      }
    } else if (r1 == r0) {
      if (lane == 0) {
        a.sp_ncells[s] = 0; a.sp_first[s] = 0; a.sp_last[s] = -1;
        a.sp_ovf_cell[s] = -1; a.sp_q1[s] = -1; a.sp_q1_shift[s] = 0;
      }
    } else if (!assemble_walk_pairs(a, s, r0, r1) && !assemble_walk(a, s, r0, r1)) {
      __threadfence_block();
      if (lane == 0) assemble_slow(a, s, r0, r1);
    }
    if (lane == 0) {
      __threadfence_block();
      assemble_finish(a, s, r1 > r0);
    }
  }
}

__global__ void __launch_bounds__(256) k_assemble(AssembleArgs a, const uint32_t* list, const uint32_t* count) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t nw = list ? *count : a.n_spans;
  for (uint32_t w = wave; w < nw; w += nwaves) assemble_span_wave(a, list ? list[w] : w);
}

}  // namespace tsdb
