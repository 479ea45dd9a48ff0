// k_ds_chunks.hip — chunk-parallel greedy downsampling for regular-cadence
// integer spans (the dominant case: series written at a fixed interval).
//
// Span.DownsamplingIterator (Span.java:377-422) chains buckets serially: a
// bucket starts at the first point >= previous start + interval. For a span
// whose first bucket holds k cells and whose cadence is regular, the heads
// are exactly the cells 0, k, 2k, ... — a hypothesis every chunk verifies
// independently for the heads it contains (head h is exact iff
// ts[h] >= ts[h-k] + interval and ts[h-1] < ts[h-k] + interval), plus the
// tail of the span's last bucket. Any miss, a float cell, a mixed-width or
// unaligned row, unsorted cells, or cells before `start` send the whole span
// to the serial kernels instead (k_decode_fast, then k_decode.hip), which
// rewrite its E sequence.
//
// Pieces: the chunk holding a bucket's head writes the head piece (count,
// timestamp sum relative to the head, integer sum/min/max); every chunk whose
// first cell is not a head writes a lead piece for the bucket open at its
// start. k_ds_finalize adds a bucket's head piece to the lead pieces of the
// chunks it spills into (integer arithmetic: exact in any order).
#pragma once
#include "dev_common.h"
#include "k_decode_fast.hip"

namespace tsdb {

struct ChunkPlanArgs {
  int32_t* row_kidx;            // [n_rows] kept index of the row's span, or -1
  const uint64_t* row_chunk0;   // [n_rows] global id of the row's first chunk
  uint32_t* plan_k;             // [n_kept] first-bucket length, 0 = not eligible
  uint32_t* plan_nb;            // [n_kept] bucket count
  uint32_t* fail;               // [n_kept] set when verification fails
  // head pieces [e_total], indexed e_off[k] + bucket
  uint32_t* hp_n;
  uint32_t* hp_ref;             // ts of the bucket head
  uint32_t* hp_rel;             // sum of (ts - head ts) over the piece
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
DEVI int64_t span_cell_ts(const DecodeArgs& a, uint64_t r0, uint64_t r1, uint32_t cell) {
  const uint64_t r = r1 - r0 == 1 ? r0 : span_cell_row(a, r0, r1, cell);
  const uint32_t q = load_qual(a.qual, a.row_qual_off[r] + 2ull * (cell - a.row_cell0[r]));
  return (int64_t)a.row_base[r] + (q >> 4);
}
DEVI uint64_t span_cell_chunk(const DecodeArgs& a, const ChunkPlanArgs& p, uint64_t r0, uint64_t r1,
                              uint32_t cell) {
  const uint64_t r = r1 - r0 == 1 ? r0 : span_cell_row(a, r0, r1, cell);
  return p.row_chunk0[r] + (cell - a.row_cell0[r]) / FCH;
}

// One wave per kept span: k = cells of the first bucket (binary search).
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
    for (uint64_t r = r0 + lane; r < r1; r += WAVE) p.row_kidx[r] = ok ? (int32_t)k : -1;
    if (lane != 0) continue;
    uint32_t kk = 0, nb = 0;
    if (ok) {
      const int64_t t0 = (int64_t)a.row_base[r0] + (load_qual(a.qual, a.row_qual_off[r0]) >> 4);
      if (t0 >= a.start) {
        const int64_t end0 = t0 + a.interval;
        uint64_t r = r0;
        for (; r < r1; r++) {
          const uint32_t nc = ncells[r];
          const int64_t last = (int64_t)a.row_base[r] + (load_qual(a.qual, a.row_qual_off[r] + 2ull * (nc - 1)) >> 4);
          if (last >= end0) break;
        }
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
        nb = kk ? (n + kk - 1) / kk : 0;
        if (kk == 0 || nb > a.sp_cap[s]) { kk = 0; nb = 0; }
      }
    }
    p.plan_k[k] = kk;
    p.plan_nb[k] = nb;
    p.fail[k] = 0;
  }
}

// One wave per row; the row's 256-cell chunks are independent (one chunk of
// loads in flight while the current one is processed).
template <int AGG>
__global__ void __launch_bounds__(256) k_ds_chunks(DecodeArgs a, ChunkPlanArgs p, const uint32_t* ncells,
                                                   const uint32_t* vlen, uint64_t n_rows) {
  constexpr bool PREFIX = AGG == 0 || AGG == 3;  // sum / avg: prefix differences; min / max: lane loops
  __shared__ uint32_t s_dt[4][FCH];
  __shared__ uint32_t s_pt[4][FCH];
  __shared__ uint64_t s_v[4][FCH];
  const int lane = lane_id();
  const int wib = threadIdx.x / WAVE;
  uint32_t* L_dt = s_dt[wib];
  uint32_t* L_pt = s_pt[wib];
  uint64_t* L_v = s_v[wib];
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / WAVE;
  for (uint64_t r = wave; r < n_rows; r += nwaves) {
    const int32_t kidx = p.row_kidx[r];
    if (kidx < 0) continue;
    const uint32_t kk = p.plan_k[kidx];
    if (kk == 0) continue;
    const uint32_t s = a.kept[kidx];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    const uint32_t ncs = a.sp_ncells[s];
    const uint32_t nb = p.plan_nb[kidx];
    const uint64_t eo = a.e_off[kidx];
    const RowMeta m = row_meta(a, r, ncells, vlen);
    bool fail = !m.ok;
    const uint32_t rcell0 = a.row_cell0[r];
    const uint64_t chunk0 = p.row_chunk0[r];
    const int64_t base = (int64_t)m.base;
    if (!fail) {
      ChunkRaw cur, nxt;
      load_chunk(a, m, 0, cur);
      for (uint32_t c0 = 0; c0 < m.nc; c0 += FCH) {
        if (c0 + FCH < m.nc) load_chunk(a, m, c0 + FCH, nxt);
        const uint32_t nv = min((uint32_t)FCH, m.nc - c0);
        const uint32_t cs = rcell0 + c0;  // span cell index of the chunk start
        // ---- decode ----
        uint32_t dt[4];
        int64_t bits[4];
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const bool valid = c0 + 4 * lane + j < m.nc;
          const uint32_t q = qual_j(cur, j);
          dt[j] = q >> 4;
          bits[j] = valid ? value_j(cur, j, m.w, false) : 0;
          bad |= valid && (((q & 7) + 1) != m.w || (q & 8) != 0);  // width, float cell
          if (j > 0) bad |= valid && dt[j] <= dt[j - 1];          // sorted within the lane
        }
        bad |= lane > 0 && 4u * lane < nv && dt[0] <= shfl_up_u32(dt[3], 1);
        // ---- stage: ts deltas, ts prefix, value prefix (or raw values) ----
        uint32_t pt = 0;
        uint64_t pv = 0;
        uint32_t pti[4];
        uint64_t pvi[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const bool valid = c0 + 4 * lane + j < m.nc;
          pt += valid ? dt[j] : 0u;
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
        // the first cell follows the previous one (previous chunk / row)
        if (lane == 0 && cs > 0) bad |= span_cell_ts(a, r0, r1, cs - 1) >= base + (int64_t)L_dt[0];
        // ---- heads n*kk inside [cs, cs+nv) ----
        const uint32_t n_lo = (cs + kk - 1) / kk;
        const uint32_t hfirst = n_lo * kk;
        const uint32_t nh = hfirst >= cs + nv ? 0u : (cs + nv - 1 - hfirst) / kk + 1;
        bad |= nh > WAVE;
        const bool mine = (uint32_t)lane < nh && nh <= WAVE;
        const uint32_t H = hfirst + (uint32_t)lane * kk;
        if (mine && H > 0) {
          // H is the first cell at/after ts[H-kk] + interval (Span.java:389-398)
          const uint32_t P = H - kk;
          const int64_t tP = P >= cs ? base + (int64_t)L_dt[P - cs] : span_cell_ts(a, r0, r1, P);
          const int64_t tH = base + (int64_t)L_dt[H - cs];
          const int64_t tH1 = H - 1 >= cs ? base + (int64_t)L_dt[H - 1 - cs] : span_cell_ts(a, r0, r1, H - 1);
          const int64_t endP = tP + a.interval;
          bad |= !(tH >= endP && tH1 < endP);
        }
        if (lane == 0 && cs + nv == ncs) {  // the last bucket holds the span's tail
          const uint32_t Hl = (nb - 1) * kk;
          const int64_t tHl = Hl >= cs ? base + (int64_t)L_dt[Hl - cs] : span_cell_ts(a, r0, r1, Hl);
          bad |= !(base + (int64_t)L_dt[nv - 1] < tHl + a.interval);
        }
        if (ballot(bad)) { fail = true; break; }
        // ---- pieces ----
        if (mine) {
          const int la = (int)(H - cs);
          const int lb = (int)min(cs + nv, H + kk) - 1 - (int)cs;
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
          const uint64_t e = eo + H / kk;
          p.hp_n[e] = n;
          p.hp_ref[e] = (uint32_t)(base + dta);
          p.hp_rel[e] = rel;
          p.hp_v[e] = v;
        }
        if (lane == 0 && hfirst != cs) {  // lead piece: cells before the first head
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
          p.lp_ts[cid] = (uint64_t)(lb + 1) * (uint64_t)m.base + L_pt[lb];
          p.lp_v[cid] = v;
        }
        wave_lds_sync();
        cur = nxt;
      }
    }
    if (fail && lane == 0) atomicOr(&p.fail[kidx], 1u);
  }
}

// One wave per verified span, one lane per bucket.
template <int AGG>
__global__ void __launch_bounds__(256) k_ds_finalize(DecodeArgs a, ChunkPlanArgs p) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  bool any = false;
  for (uint32_t k = wave; k < a.n_kept; k += nwaves) {
    const uint32_t kk = p.plan_k[k];
    if (kk == 0 || p.fail[k]) continue;
    const uint32_t nb = p.plan_nb[k];
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    const uint32_t ncs = a.sp_ncells[s];
    const uint64_t eo = a.e_off[k];
    for (uint32_t b = lane; b < nb; b += WAVE) {
      uint32_t n = p.hp_n[eo + b];
      const int64_t ref = p.hp_ref[eo + b];
      uint64_t rel = p.hp_rel[eo + b];
      int64_t v = p.hp_v[eo + b];
      const uint32_t H = b * kk;
      const uint32_t last = min(ncs, H + kk) - 1;
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
  if (p.plan_k[k] == 0 || p.fail[k]) p.list[atomicAdd(p.list_count, 1u)] = k;
}

__global__ void k_row_chunks(const uint32_t* ncells, uint64_t n_rows, uint64_t* out) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n_rows) out[r] = (ncells[r] + FCH - 1) / FCH;
}

}  // namespace tsdb
