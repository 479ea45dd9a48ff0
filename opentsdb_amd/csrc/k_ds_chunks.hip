// k_ds_chunks.hip — chunk-parallel greedy downsampling for regular-cadence
// integer spans (the dominant case: series written at a fixed interval).
//
// Span.DownsamplingIterator (Span.java:377-422) chains buckets serially: a
// bucket starts at the first point >= previous start + interval. For a span
// whose first bucket holds k cells and whose cadence is regular, the heads
// are exactly the cells 0, k, 2k, ... The chunk kernel assumes that and
// records, per head h, ts[h] and ts[h-1]; k_ds_finalize then proves it:
// head h is exact iff ts[h] >= ts[h-k] + interval > ts[h-1], and the span's
// last cell must stay inside the last bucket. Any miss, a float cell, a
// mixed-width or unaligned row, unsorted cells, or cells before `start`
// send the whole span to the serial kernels instead (k_decode_fast, then
// k_decode.hip), which rewrite its E sequence.
//
// Pieces: the chunk holding a bucket's head writes the head piece (count,
// timestamp sum relative to the head, integer sum/min/max); every chunk whose
// first cell is not a head writes a lead piece for the bucket open at its
// start. k_ds_finalize adds a bucket's head piece to the lead pieces of the
// chunks it spills into (integer arithmetic: exact in any order).
//
// The chunk loop issues no global load besides the chunk stream itself: an
// in-order vmcnt wait for any other load would also drain the prefetched
// chunks.
#pragma once
#include "dev_common.h"
#include "k_decode_fast.hip"

namespace tsdb {

struct alignas(16) SpanPlan {
  uint32_t kk;    // first-bucket length in cells, 0 = not eligible
  uint32_t nb;    // bucket count
  uint32_t ncs;   // span cells
  uint32_t pad;
  uint64_t eo;    // E offset
  uint64_t r0;    // first row
};

struct ChunkPlanArgs {
  int32_t* row_kidx;            // [n_rows] kept index of the row's span, or -1
  uint32_t* row_prev_ts;        // [n_rows] last ts of the previous row of the span
  const uint64_t* row_chunk0;   // [n_rows] global id of the row's first chunk
  SpanPlan* plan;               // [n_kept]
  uint32_t* fail;               // [n_kept] set when verification fails
  uint32_t* tail_ts;            // [n_kept] ts of the span's last cell
  // head pieces [e_total], indexed e_off[k] + bucket
  uint32_t* hp_nrel;            // n << 20 | sum of (ts - head ts) (n <= 256, sum < 2^20)
  uint32_t* hp_ref;             // ts of the head
  uint32_t* hp_pre;             // ts of the cell before the head
  int64_t* hp_v;                // integer sum / min / max of the piece
  // lead pieces [n_chunks]
  uint32_t* lp_n;
  uint64_t* lp_ts;              // absolute timestamp sum
  int64_t* lp_v;
  uint32_t* list;               // spans for the serial kernels
  uint32_t* list_count;
};

// last row of [r0, r1) whose first span cell is <= cell
DEVI uint64_t span_cell_row(const DecodeArgs& a, uint64_t r0, uint64_t r1, uint32_t cell) {
  uint64_t lo = r0, hi = r1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a.row_cell0[mid] <= cell) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}
DEVI uint64_t span_cell_chunk(const DecodeArgs& a, const ChunkPlanArgs& p, uint64_t r0, uint64_t r1,
                              uint32_t cell) {
  const uint64_t r = r1 - r0 == 1 ? r0 : span_cell_row(a, r0, r1, cell);
  return p.row_chunk0[r] + (cell - a.row_cell0[r]) / FCH;
}
DEVI uint32_t row_last_ts(const DecodeArgs& a, uint64_t r, const uint32_t* ncells) {
  return a.row_base[r] + (load_qual(a.qual, a.row_qual_off[r] + 2ull * (ncells[r] - 1)) >> 4);
}

// One wave per kept span: eligibility, k = cells of the first bucket.
__global__ void __launch_bounds__(256) k_ds_plan(DecodeArgs a, ChunkPlanArgs p, const uint32_t* ncells) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  for (uint32_t k = wave; k < a.n_kept; k += nwaves) {
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    const uint32_t n = a.sp_ncells[s];
    bool ok = a.sp_q1[s] < 0 && a.sp_ovf_cell[s] < 0 && n > 0 && r1 > r0;
    for (uint64_t r = r0 + lane; r < r1 + lane; r += WAVE)
      ok &= ballot(r < r1 && (a.row_ok[r] == 0 || ncells[r] == 0)) == 0;
    for (uint64_t r = r0 + lane; r < r1; r += WAVE) {
      p.row_kidx[r] = ok ? (int32_t)k : -1;
      if (ok && r > r0) p.row_prev_ts[r] = row_last_ts(a, r - 1, ncells);
    }
    // common case: the first bucket ends within the first row's first 64 cells
    int probe = -1;  // first probed cell at/after t0 + interval
    int64_t t0 = 0;
    if (ok) {
      const uint32_t nc0 = ncells[r0];
      const uint64_t qo = a.row_qual_off[r0];
      const int64_t b0 = (int64_t)a.row_base[r0];
      t0 = b0 + (load_qual(a.qual, qo) >> 4);
      const bool in = (uint32_t)lane < nc0;
      const int64_t t = in ? b0 + (load_qual(a.qual, qo + 2ull * lane) >> 4) : 0;
      const uint64_t hit = ballot(in && t >= t0 + a.interval);
      if (hit) probe = __builtin_ctzll(hit);
    }
    if (lane != 0) continue;
    uint32_t kk = 0, nb = 0;
    if (ok && t0 >= a.start) {
      const int64_t end0 = t0 + a.interval;
      if (probe > 0) {
        kk = (uint32_t)probe;
      } else {
        uint64_t r = r0;
        for (; r < r1; r++)
          if ((int64_t)row_last_ts(a, r, ncells) >= end0) break;
        if (r == r1) {
          kk = n;  // one bucket holds the whole span
        } else {
          uint32_t lo = 0, hi = ncells[r];
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const int64_t t = (int64_t)a.row_base[r] + (load_qual(a.qual, a.row_qual_off[r] + 2ull * mid) >> 4);
            if (t < end0) lo = mid + 1; else hi = mid;
          }
          kk = a.row_cell0[r] + lo;
        }
      }
      nb = kk ? (n + kk - 1) / kk : 0;
      if (kk == 0 || nb > a.sp_cap[s]) { kk = 0; nb = 0; }
    }
    SpanPlan sp;
    sp.kk = kk; sp.nb = nb; sp.ncs = n; sp.pad = 0; sp.eo = a.e_off[k]; sp.r0 = r0;
    p.plan[k] = sp;
    p.fail[k] = 0;
  }
}

template <int W>
struct RawW {
  uint2 q;             // 4 big-endian qualifiers
  uint4 v[W / 4];      // 4 values
};

// Branch-free chunk load; c is clamped into the row by the caller. Reads up
// to 3 cells past the row end (inside the buffers' 64-byte slack).
template <int W>
DEVI void load_raw(const DecodeArgs& a, uint64_t qoff, uint64_t voff, uint32_t c, RawW<W>& x) {
  x.q = *(const uint2*)(a.qual + qoff + 2ull * c);
  const uint4* pv = (const uint4*)(a.val + voff + (uint64_t)W * c);
#pragma unroll
  for (int i = 0; i < W / 4; i++) x.v[i] = pv[i];
}

template <int W>
DEVI int64_t raw_value(const RawW<W>& x, int j) {
  if (W == 8) {
    const uint4 u = x.v[j >> 1];
    const uint32_t lo = (j & 1) ? u.z : u.x, hi = (j & 1) ? u.w : u.y;
    return (int64_t)bswap64((uint64_t)lo | ((uint64_t)hi << 32));
  }
  const uint4 u = x.v[0];
  const uint32_t w = j == 0 ? u.x : j == 1 ? u.y : j == 2 ? u.z : u.w;
  return (int64_t)(int32_t)bswap32(w);
}

DEVI uint32_t raw_qual(uint2 q, int j) {
  const uint32_t word = j < 2 ? q.x : q.y;
  const uint32_t h = (j & 1) ? (word >> 16) : (word & 0xFFFF);
  return ((h & 0xFF) << 8) | (h >> 8);
}

// One row: its 256-cell chunks, two chunks of loads in flight. Returns true
// if the row breaks a precondition (the span then goes to the serial path).
template <int AGG, int W>
DEVI bool chunk_row(const DecodeArgs& a, const ChunkPlanArgs& p, const SpanPlan& sp, uint32_t kidx,
                    uint64_t qoff, uint64_t voff, uint32_t base, uint32_t nc, uint32_t cell0, uint64_t chunk0,
                    bool has_prev, uint32_t prev_ts, uint32_t* L_dt, uint32_t* L_pt, uint64_t* L_v) {
  constexpr bool PREFIX = AGG == 0 || AGG == 3;  // sum / avg: prefix differences; min / max: lane loops
  const int lane = lane_id();
  const uint32_t kk = sp.kk;
  const uint32_t clamp_c = (nc - 1) & ~3u;
  // three register sets; the loop is unrolled by 3 so their roles rotate
  // statically (a register copy of an in-flight load would wait for it)
  RawW<W> A, B, C;
  auto issue = [&](uint32_t c0, RawW<W>& x) {
    const uint32_t c = c0 + 4u * lane;
    load_raw<W>(a, qoff, voff, c < nc ? c : clamp_c, x);
  };
  issue(0, A);
  issue(FCH, B);
  uint32_t bfirst = (cell0 + kk - 1) / kk;  // first bucket whose head is at/after the row start
  uint32_t hfirst = bfirst * kk;
  bool bad = false;
  // process chunk c0 held in `cur`
  auto step = [&](uint32_t c0, const RawW<W>& cur) {
    const uint32_t nv = min((uint32_t)FCH, nc - c0);
    const uint32_t cs = cell0 + c0;  // span cell index of the chunk start
    // ---- decode ----
    uint32_t dt[4];
    int64_t bits[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const bool valid = 4u * lane + j < nv;
      const uint32_t q = raw_qual(cur.q, j);
      dt[j] = valid ? q >> 4 : 0u;
      bits[j] = valid ? raw_value<W>(cur, j) : 0;
      bad |= valid && (q & 15) != (uint32_t)(W - 1);  // integer cell of this width
      if (j > 0) bad |= valid && dt[j] <= dt[j - 1];  // sorted within the lane
    }
    {
      const uint32_t pl = shfl_up_u32(dt[3], 1);
      bad |= lane > 0 && 4u * lane < nv && dt[0] <= pl;
      bad |= lane == 0 && has_prev && base + dt[0] <= prev_ts;  // previous chunk / row
    }
    // ---- stage: ts deltas, ts prefix, value prefix (or raw values) ----
    uint32_t pt = 0;
    uint64_t pv = 0;
    uint32_t pti[4];
    uint64_t pvi[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      pt += dt[j];
      pv += (uint64_t)bits[j];
      pti[j] = pt;
      pvi[j] = PREFIX ? pv : (uint64_t)bits[j];
    }
    const uint32_t xt = wave_incl_scan_u32_dpp(pt) - pt;
    *(uint4*)&L_pt[4 * lane] = make_uint4(pti[0] + xt, pti[1] + xt, pti[2] + xt, pti[3] + xt);
    *(uint4*)&L_dt[4 * lane] = make_uint4(dt[0], dt[1], dt[2], dt[3]);
    {
      const uint64_t xv = PREFIX ? wave_incl_scan_u64_dpp(pv) - pv : 0ull;
      ulonglong2 v01, v23;
      v01.x = pvi[0] + xv; v01.y = pvi[1] + xv; v23.x = pvi[2] + xv; v23.y = pvi[3] + xv;
      *(ulonglong2*)&L_v[4 * lane] = v01;
      *(ulonglong2*)&L_v[4 * lane + 2] = v23;
    }
    wave_lds_sync();
    // ---- heads: lane j owns head hfirst + j*kk if it lies in the chunk ----
    const uint64_t H64 = (uint64_t)hfirst + (uint64_t)lane * kk;
    const bool mine = H64 < (uint64_t)cs + nv;
    const uint64_t hm = ballot(mine);
    bad |= hm == ~0ull;  // 64+ heads in one chunk: one lane per head cannot hold them
    const uint32_t nh = (uint32_t)__builtin_popcountll(hm);
    if (mine) {
      const uint32_t H = (uint32_t)H64;
      const int la = (int)(H - cs);
      const int lb = (int)(min((uint64_t)cs + nv, H64 + kk) - 1 - cs);
      const uint32_t n = (uint32_t)(lb - la + 1);
      const uint32_t dta = L_dt[la];
      const uint32_t rel = (L_pt[lb] - (la > 0 ? L_pt[la - 1] : 0u)) - n * dta;
      int64_t v;
      if (PREFIX) {
        v = (int64_t)(L_v[lb] - (la > 0 ? L_v[la - 1] : 0ull));
      } else {
        v = (int64_t)L_v[la];
        for (int i = la + 1; i <= lb; i++) {
          const int64_t x = (int64_t)L_v[i];
          if (AGG == 1 ? x < v : x > v) v = x;
        }
      }
      const uint64_t e = sp.eo + bfirst + (uint32_t)lane;
      p.hp_nrel[e] = (n << 20) | rel;
      p.hp_ref[e] = base + dta;
      p.hp_pre[e] = la > 0 ? base + L_dt[la - 1] : prev_ts;
      p.hp_v[e] = v;
    }
    const uint32_t last_ts = base + L_dt[nv - 1];
    if (lane == 0) {
      if (hfirst != cs) {  // lead piece: cells before the chunk's first head
        const int lb = nh > 0 ? (int)(hfirst - cs) - 1 : (int)nv - 1;
        int64_t v;
        if (PREFIX) {
          v = (int64_t)L_v[lb];
        } else {
          v = (int64_t)L_v[0];
          for (int i = 1; i <= lb; i++) {
            const int64_t x = (int64_t)L_v[i];
            if (AGG == 1 ? x < v : x > v) v = x;
          }
        }
        const uint64_t cid = chunk0 + c0 / FCH;
        p.lp_n[cid] = (uint32_t)(lb + 1);
        p.lp_ts[cid] = (uint64_t)(lb + 1) * (uint64_t)base + L_pt[lb];
        p.lp_v[cid] = v;
      }
      if (cs + nv == sp.ncs) p.tail_ts[kidx] = last_ts;
    }
    prev_ts = last_ts;
    has_prev = true;
    hfirst += nh * kk;
    bfirst += nh;
    wave_lds_sync();
  };
  // loads past the row end are clamped (cache hits); steps past it skipped
  for (uint32_t c0 = 0; c0 < nc; c0 += 3 * FCH) {
    issue(c0 + 2 * FCH, C);
    step(c0, A);
    issue(c0 + 3 * FCH, A);
    if (c0 + FCH < nc) step(c0 + FCH, B);
    issue(c0 + 4 * FCH, B);
    if (c0 + 2 * FCH < nc) step(c0 + 2 * FCH, C);
  }
  return ballot(bad) != 0;
}

// One wave per row.
template <int AGG>
__global__ void __launch_bounds__(256) k_ds_chunks(DecodeArgs a, ChunkPlanArgs p, const uint32_t* ncells,
                                                   const uint32_t* vlen, uint64_t n_rows) {
  __shared__ uint32_t s_dt[4][FCH];
  __shared__ uint32_t s_pt[4][FCH];
  __shared__ uint64_t s_v[4][FCH];
  const int lane = lane_id();
  const int wib = threadIdx.x / WAVE;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / WAVE;
  for (uint64_t r = wave; r < n_rows; r += nwaves) {
    const int32_t kidx = p.row_kidx[r];
    if (kidx < 0) continue;
    const SpanPlan sp = p.plan[kidx];
    if (sp.kk == 0) continue;
    const uint32_t nc = ncells[r];
    const uint32_t vl = vlen[r];
    const uint64_t qoff = a.row_qual_off[r], voff = a.row_val_off[r];
    const uint32_t vb = nc > 1 ? vl - 1 : vl;
    const uint32_t w = vb / nc;
    const bool aligned = vb == w * nc && (qoff & 7) == 0 && (voff & 15) == 0;
    const bool first = r == sp.r0;
    const uint32_t prev_ts = first ? 0u : p.row_prev_ts[r];
    bool fail = true;
    if (aligned && w == 8)
      fail = chunk_row<AGG, 8>(a, p, sp, (uint32_t)kidx, qoff, voff, a.row_base[r], nc, a.row_cell0[r],
                               p.row_chunk0[r], !first, prev_ts, s_dt[wib], s_pt[wib], s_v[wib]);
    else if (aligned && w == 4)
      fail = chunk_row<AGG, 4>(a, p, sp, (uint32_t)kidx, qoff, voff, a.row_base[r], nc, a.row_cell0[r],
                               p.row_chunk0[r], !first, prev_ts, s_dt[wib], s_pt[wib], s_v[wib]);
    if (fail && lane == 0) atomicOr(&p.fail[kidx], 1u);
  }
}

// One wave per eligible span, one lane per bucket: proves the heads, then
// combines the pieces into E.
template <int AGG>
__global__ void __launch_bounds__(256) k_ds_finalize(DecodeArgs a, ChunkPlanArgs p) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  bool any = false;
  for (uint32_t k = wave; k < a.n_kept; k += nwaves) {
    const SpanPlan sp = p.plan[k];
    if (sp.kk == 0 || p.fail[k]) continue;
    const uint32_t kk = sp.kk, nb = sp.nb;
    const uint64_t eo = sp.eo;
    const uint64_t r0 = sp.r0, r1 = a.span_row_start[a.kept[k] + 1];
    const int64_t I = a.interval;
    bool bad = false;
    for (uint32_t b = lane; b < nb; b += WAVE) {
      const uint32_t nrel = p.hp_nrel[eo + b];
      uint32_t n = nrel >> 20;
      uint64_t rel = nrel & 0xFFFFFu;
      const int64_t ref = p.hp_ref[eo + b];
      int64_t v = p.hp_v[eo + b];
      if (b > 0) {  // Span.java:389-398: the head is the first cell at/after the previous end
        const int64_t end = (int64_t)p.hp_ref[eo + b - 1] + I;
        bad |= !(ref >= end && (int64_t)p.hp_pre[eo + b] < end);
      }
      if (b == nb - 1) bad |= !((int64_t)p.tail_ts[k] < ref + I);
      const uint32_t H = b * kk;
      const uint32_t last = min(sp.ncs, H + kk) - 1;
      if (last >= H + n) {  // the bucket spills into the following chunks
        const uint64_t c_first = span_cell_chunk(a, p, r0, r1, H + n);
        const uint64_t c_last = span_cell_chunk(a, p, r0, r1, last);
        for (uint64_t c = c_first; c <= c_last; c++) {
          const uint32_t ln = p.lp_n[c];
          rel += p.lp_ts[c] - (uint64_t)ln * (uint64_t)ref;
          n += ln;
          const int64_t x = p.lp_v[c];
          if (AGG == 0 || AGG == 3) v = ladd(v, x);
          else if (AGG == 1 ? x < v : x > v) v = x;
        }
      }
      a.e_ts[eo + b] = (uint32_t)(ref + (int64_t)udiv64_32(rel, n));  // Span.java:399
      a.e_val[eo + b] = AGG == 3 ? ldiv64_32(v, n) : v;
      a.e_flt[eo + b] = 0;
    }
    if (ballot(bad)) {  // not the greedy chain: the serial kernels rewrite this span
      if (lane == 0) p.fail[k] = 1;
      continue;
    }
    if (lane == 0) {
      a.e_len[k] = nb;
      a.e_bad[k] = -1;
    }
    any = true;
  }
  if (any && lane == 0 && !a.gflags[1]) atomicOr(&a.gflags[1], 1u);
}

// Spans not eligible or failing verification -> the serial kernels.
__global__ void k_ds_collect(DecodeArgs a, ChunkPlanArgs p) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.n_kept) return;
  if (p.plan[k].kk == 0 || p.fail[k]) p.list[atomicAdd(p.list_count, 1u)] = k;
}

__global__ void k_row_chunks(const uint32_t* ncells, uint64_t n_rows, uint64_t* out) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n_rows) out[r] = (ncells[r] + FCH - 1) / FCH;
}

}  // namespace tsdb
