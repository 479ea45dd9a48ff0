// k_ds_reg.hip — greedy downsampling of constant-step spans by formula: the
// first pass over a downsampled SpanGroup's kept spans.
//
// Span.DownsamplingIterator (Span.java:377-422) chains buckets serially: a
// bucket starts at the first point at/after the previous start + interval.
// On a span whose cells sit at ts = t0 + c * step (c = span cell index, every
// cell, every row), the chain is closed-form: kk = ceil(interval / step) cells
// per bucket, heads at c = 0, kk, 2kk, ..., so bucket b holds cells
// [b kk, min((b+1) kk, n)) and its timestamp ⌊Σts / m⌋ (Span.java:399) is
// t0 + b kk step + ⌊step (m - 1) / 2⌋ (m cells) — no chain proof, no
// timestamp scan, no division. The wave proves the premise instead: each
// lane compares its 8 qualifiers with the expected ones ((t0 + c step - base)
// << 4 | flags, one xor per pair of cells), and each row's first / last delta
// lies in [0, 4095]. Buckets close inside the chunk that holds their last
// cell; value sums are differences of an LDS prefix (exact, wrapping), double
// buckets (and min / max) a lane per bucket in point order
// (Aggregators.java:86-180). The bucket still open at the end of a chunk is
// carried in a wave-uniform register.
//
// The bucket heads being known up front, a span of many rows (C2: 24 hourly
// rows of 360 cells) is split over up to 4 waves of one block, each taking a
// contiguous run of rows that starts at a bucket head; the waves agree on the
// span's fate at one block barrier before its grid points are marked.
// Anything else — a cadence break, mixed widths or types, a first cell before
// `start`, a piece boundary inside a bucket, dropped rows, Q1 / short
// overflow — sends the whole span to k_ds_spans (chain-proved cadence), and
// from there to the serial kernels, which rewrite its E.
#pragma once
#include "dev_common.h"
#include "k_ds_chunks.hip"

namespace tsdb {

// x / d for u32 x by one multiply-high (round-up magic number, exact for
// every u32 x; Granlund & Montgomery): set up once per span, wave-uniform.
struct UDiv {
  uint32_t m, s1, s2;
  DEVI void init(uint32_t d) {
    if (d == 1) { m = 0; s1 = 0; s2 = 0; return; }
    const uint32_t l = 32 - __clz(d - 1);
    m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d) + 1;
    s1 = 1;
    s2 = l - 1;
  }
  DEVI uint32_t div(uint32_t x) const {
    const uint32_t t = __umulhi(x, m);
    return (t + ((x - t) >> s1)) >> s2;
  }
};

// wave-uniform description of a constant-step span
struct RegSpan {
  uint32_t t0, step, kk, n;  // first ts, cadence, cells per bucket, cells
  uint64_t eo;               // E offset
  uint32_t cap;              // E capacity
  UDiv dkk;                  // / kk
};

// E entries of buckets [b0, b0 + cnt) (cnt <= 64) from the per-wave bucket
// buffer (their values over their cells; timestamps by formula): one lane per
// bucket, so the avg divisions (Span.java:399-420 with Aggregators.Avg)
// leave the chunk loop.
// fop >= 0 (an aligned group, FapArgs): integer bucket values go into the
// block's partial per bucket index instead (the cross-series aggregator's
// combine: 0 wrapping add, 1 min, 2 max), no E.
template <int AGG, bool FLT>
DEVI void reg_flush(const DecodeArgs& a, const RegSpan& sp, const int64_t* BK, uint32_t b0, uint32_t cnt, int fop,
                    int64_t* part) {
  wave_lds_sync();
  const uint32_t i = lane_id();
  if (!FLT && fop >= 0) {
    if (i < cnt) {
      const uint32_t b = b0 + i;
      const uint32_t sb = b * sp.kk, m = min(sb + sp.kk, sp.n) - sb;
      const int64_t v = AGG == 3 ? ldiv64_32(BK[i], m) : BK[i];
      if (fop == 0) atomicAdd((unsigned long long*)&part[b], (unsigned long long)v);
      else if (fop == 1) atomicMin((long long*)&part[b], (long long)v);
      else atomicMax((long long*)&part[b], (long long)v);
    }
    wave_lds_sync();
    return;
  }
  if (i < cnt) {
    const uint32_t b = b0 + i;
    const uint32_t sb = b * sp.kk, m = min(sb + sp.kk, sp.n) - sb;
    const int64_t v = BK[i];
    const uint64_t o = sp.eo + b;
    // (fop -2, the uniform path's E variant: values only, the timestamps
    // being G and the type the key's)
    if (fop != -2) a.e_ts[o] = sp.t0 + sb * sp.step + (uint32_t)((uint64_t)sp.step * (m - 1) / 2);
    if (FLT)  // Aggregators.Avg.runDouble: sum / n
      a.e_val[o] = AGG == 3 ? dbits(bitsd(v) / (double)(int32_t)m) : v;
    else
      a.e_val[o] = AGG == 3 ? ldiv64_32(v, m) : v;
    if (fop != -2) a.e_flt[o] = FLT ? 1 : 0;
  }
  wave_lds_sync();
}

// L_v's layout: lane l stages cells 8 l .. 8 l + 7 as four 16-B pairs, pair
// p at slot (p + (l >> 1)) & 3 of the lane's 64 bytes, so the 8 lanes of a
// ds_write_b128 group hit 8 distinct 16-B bank quads (the
// unrotated 64-B lane stride cost 15.6 conflict cycles an LDS instruction on
// C2); cell c sits at lv_ix(c).
DEVI uint32_t lv_ix(uint32_t c) {
  const uint32_t l = c >> 3;
  return (l << 3) | (((((c >> 1) & 3u) + (l >> 1)) & 3u) << 1) | (c & 1u);
}

// The chunks of rows [ra, rb) of one span (two register sets, the next
// chunk's loads in flight while one is processed, as ds_span); buckets that
// close in these rows go to E. Returns true if the premise breaks. The
// caller checked the rows (reg_rows_ok) and that ra starts a bucket.
template <int AGG, int W, bool FLT>
DEVI bool reg_piece(const DecodeArgs& a, const RegSpan& sp, uint64_t ra, uint64_t rb, const uint32_t* ncells,
                    uint64_t* L_v, int64_t* BK, int fop, int64_t* part) {
  constexpr bool PREFIX = (AGG == 0 || AGG == 3) && !FLT;  // wrapping sums: prefix differences
  const int lane = lane_id();
  const uint32_t fl = (FLT ? 8u : 0u) | (uint32_t)(W - 1);
  const uint32_t nb = sp.dkk.div(sp.n + sp.kk - 1);
  auto row_at = [&](uint64_t r) {
    ChunkPos p;
    p.r = r;
    p.nc = sld(&ncells[r]);
    p.qoff = sld(&a.row_qual_off[r]);
    p.voff = sld(&a.row_val_off[r]);
    p.base = sld(&a.row_base[r]);
    p.cell0 = sld(&a.row_cell0[r]);
    p.c0 = 0;
    p.done = false;
    return p;
  };
  auto advance = [&](const ChunkPos& p) {
    if (p.done) return p;
    if (p.c0 + DCH < p.nc) {
      ChunkPos q = p;
      q.c0 += DCH;
      return q;
    }
    if (p.r + 1 < rb) return row_at(p.r + 1);
    ChunkPos q = p;
    q.done = true;
    return q;
  };
  RawW<W> A, B;
  auto issue = [&](const ChunkPos& p, RawW<W>& x) {
    const uint32_t c = p.c0 + 8u * lane;
    __builtin_amdgcn_s_setprio(2);
    load_raw<W>(a, p.qoff, p.voff, c < p.nc ? c : (p.nc - 1) & ~7u, x);
    __builtin_amdgcn_s_setprio(0);
  };
  bool bad = false;
  int64_t carry = 0;  // the open bucket's value over its cells in earlier chunks
  // bucket of the next chunk's first cell and that cell's place in it
  uint32_t bcur = sp.dkk.div(sld(&a.row_cell0[ra])), ph = 0;
  uint32_t fbase = bcur;  // first bucket held in BK
  uint32_t bclosed = bcur;  // buckets closed so far: [.., bclosed)
  // decode + qualifier check + LDS staging of one chunk (FULL: 512 cells)
  auto stage = [&](auto full, const ChunkPos& p, const RawW<W>& cur, uint32_t nv, uint32_t cs) {
    constexpr bool FULL = decltype(full)::value;
    const uint32_t nmine = FULL ? 8u : (nv > 8u * lane ? min(8u, nv - 8u * lane) : 0u);
    {  // (t0 + c step - base) << 4 | flags, two cells per dword
      const uint32_t d0 = sp.t0 + (cs + 8u * lane) * sp.step - p.base;
      uint32_t e = ((d0 << 4) | fl) * 0x00010001u + (sp.step << 20);
      const uint32_t inc = sp.step * 0x00200020u;
      const uint32_t qw[4] = {cur.q.x, cur.q.y, cur.q.z, cur.q.w};
      uint32_t miss = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        uint32_t x = qpair(qw[i]) ^ e;
        if (!FULL) x &= nmine >= 2u * i + 2 ? 0xFFFFFFFFu : (nmine == 2u * i + 1 ? 0x0000FFFFu : 0u);
        miss |= x;
        e += inc;
      }
      bad |= miss != 0;
    }
    int64_t bits[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      bits[j] = raw_value<W>(cur, j);
      if (W == 4 && FLT) bits[j] = dbits((double)__int_as_float((int32_t)bits[j]));
      if (!FULL && (uint32_t)j >= nmine) bits[j] = 0;
    }
    uint64_t pv = 0, pvi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      pv += (uint64_t)bits[j];
      pvi[j] = PREFIX ? pv : (uint64_t)bits[j];
    }
    const uint64_t xv = PREFIX ? wave_incl_scan_u64_dpp(pv) - pv : 0ull;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      ulonglong2 v2;
      v2.x = pvi[j] + xv;
      v2.y = pvi[j + 1] + xv;
      *(ulonglong2*)&L_v[8 * lane + 2 * (((uint32_t)(j >> 1) + ((uint32_t)lane >> 1)) & 3u)] = v2;
    }
  };
  auto step = [&](const ChunkPos& p, const RawW<W>& cur) {
    const uint32_t nv = ufl(min(DCH, p.nc - p.c0));
    const uint32_t cs = ufl(p.cell0 + p.c0);  // span cell index of the chunk start
    if (nv == DCH) stage(std::integral_constant<bool, true>(), p, cur, nv, cs);
    else stage(std::integral_constant<bool, false>(), p, cur, nv, cs);
    wave_lds_sync();
    // ---- buckets ending in [cs, cend), then the one still open at cend ----
    const uint32_t cend = cs + nv;
    const uint32_t kk = sp.kk;
    const uint32_t adv = sp.dkk.div(ph + nv);  // buckets whose last cell is in the chunk (full ones)
    const uint32_t b_lo = bcur;
    const uint32_t b_end = cend == sp.n ? nb : b_lo + adv;  // first bucket not closed here
    ph = ph + nv - adv * kk;
    bcur = b_lo + adv;
    const bool open = cend < sp.n && ph != 0;  // bucket b_end takes later cells
    const uint32_t nclose = b_end - b_lo;
    bclosed = b_end;
    const uint32_t ntot = nclose + (open ? 1u : 0u);
    int64_t carry_next = 0;
    for (uint32_t jb = 0; jb < ntot; jb += WAVE) {
      const uint32_t j = jb + lane;
      const bool act = j < ntot;
      const uint32_t b = b_lo + (act ? j : 0u);
      const uint32_t sb = b * kk;
      const uint32_t eb = act && j < nclose ? min(sb + kk, sp.n) - 1 : cend - 1;  // (open: its cells so far)
      const uint32_t la = sb > cs ? sb - cs : 0u, lb = eb - cs;
      const bool cont = sb < cs;  // began in an earlier chunk
      int64_t v;
      if (PREFIX) {
        v = (int64_t)(L_v[lv_ix(lb)] - (la > 0 ? L_v[lv_ix(la - 1)] : 0ull));
        if (cont) v = ladd(v, carry);
      } else if (FLT) {
        double d = cont ? bitsd(carry) : bitsd((int64_t)L_v[lv_ix(la)]);
        for (uint32_t i = cont ? la : la + 1; act && i <= lb; i++) d = ds_dcombine<AGG>(d, bitsd((int64_t)L_v[lv_ix(i)]));
        v = dbits(d);
      } else {
        v = cont ? carry : (int64_t)L_v[lv_ix(la)];
        for (uint32_t i = cont ? la : la + 1; act && i <= lb; i++) v = ds_combine<AGG>(v, (int64_t)L_v[lv_ix(i)]);
      }
      // closed buckets -> the bucket buffer (room for this pass's first)
      const uint32_t pc = min(nclose - min(nclose, jb), (uint32_t)WAVE);
      if (pc) {
        if (b_lo + jb + pc - fbase > WAVE) {
          reg_flush<AGG, FLT>(a, sp, BK, fbase, b_lo + jb - fbase, fop, part);
          fbase = b_lo + jb;
        }
        if (act && j < nclose) BK[b - fbase] = v;
      }
      if (open && jb + WAVE >= ntot) carry_next = (int64_t)readlane_u64((uint64_t)v, (int)(ntot - 1 - jb));
    }
    carry = carry_next;
    wave_lds_sync();
  };
  ChunkPos p0 = row_at(ra);
  ChunkPos p1 = advance(p0);
  issue(p0, A);
  issue(p1, B);
  for (;;) {
    step(p0, A);
    if (p1.done || ballot(bad) != 0) break;
    const ChunkPos p2 = advance(p1);
    issue(p2, A);
    step(p1, B);
    if (p2.done || ballot(bad) != 0) break;
    const ChunkPos p3 = advance(p2);
    issue(p3, B);
    p0 = p2;
    p1 = p3;
  }
  // the piece ends at the span's end or at a bucket boundary (else the next
  // piece does not start a bucket: the whole span is redone)
  bad |= bclosed != nb && ph != 0;
  if (ballot(bad) != 0) return true;
  if (bclosed > fbase) reg_flush<AGG, FLT>(a, sp, BK, fbase, bclosed - fbase, fop, part);
  return false;
}

// Row checks of rows [ra, rb) of a span in constant-step form: kept, cells of
// width W (value bytes = W n, + the meta byte of a compacted row), aligned,
// every delta t0 + c step - base inside [0, 4095] (monotone in c: the first
// and the last cell of the row decide).
DEVI bool reg_rows_ok(const DecodeArgs& a, const RegSpan& sp, uint64_t ra, uint64_t rb, uint32_t W) {
  const int lane = lane_id();
  bool ok = true;
  for (uint64_t rr = ra; ok && rr < rb; rr += WAVE) {  // (uniform loop: keeps `ok` scalar)
    const uint64_t r = rr + lane;
    bool rbad = false;
    if (r < rb) {
      const uint32_t nc = a.row_ncells[r], vl = a.row_val_len[r];
      const uint32_t vb = nc > 1 ? vl - 1 : vl;
      const int64_t d0 = (int64_t)sp.t0 + (int64_t)a.row_cell0[r] * sp.step - (int64_t)a.row_base[r];
      const int64_t d1 = d0 + (int64_t)(nc - 1) * sp.step;
      rbad = a.row_ok[r] == 0 || nc == 0 || vb != W * nc || (a.row_qual_off[r] & 7) != 0 ||
             (a.row_val_off[r] & 15) != 0 || d0 < 0 || d1 > 4095;
    }
    ok = ballot(rbad) == 0;
  }
  return ok;
}

// The aligned-group reduction (FAP, SURVEY.md §8(e)'s "skip the grid
// exchange when all shards agree", taken one step further): when every kept
// span of the group is a constant-step integer span with the same first ts,
// cadence and length (C3*: series written in lockstep), they share one bucket
// sequence, the union grid G is that sequence (bucket ts <= end), and every
// span is active at every t of G (SpanGroup.java:510-608), so the
// cross-series integer aggregate at G[b] is the combine of bucket b over the
// spans (wrapping sum / min / max, exact in any order; avg divides the sum by
// the span count in the finalize, Aggregators.java:76-180). Each block then
// combines its spans' buckets in LDS and writes one partial row instead of
// the spans' E; k_fap_rows / k_fap_final reduce the rows into the 1-chunk
// partial layout k_reduce would write. Any span outside the class sets
// `broken` and the host reruns k_ds_reg with `rewrite` (E for the spans it
// takes, nothing else), then reduces as usual.
struct FapArgs {
  int32_t op;        // -1: off; else 0 wrapping add (sum, avg), 1 min, 2 max
  int32_t rewrite;   // 1: the rerun after a broken FAP pass
  int64_t* part;     // [gridDim.x][64] block partials per bucket index
  unsigned long long* key;  // [4] Small.fap_key
  uint32_t* broken;         // Small.fap_broken
  uint32_t nrows;           // (host) partial rows written: the launch's blocks
  // (the uniform path) instead of a row a block: the block's partial combined
  // by device atomics into copy (block % ncopy) of 64 slots, neutral on entry
  unsigned long long* copies;
  uint32_t ncopy;
  // (the uniform path's E variant, op -1) every kept span proposed one key:
  // block 0 writes G, the key's bucket timestamps; the spans' E values only
  // (k_ug_reduce); a span the kernel does not take sets `broken` (the call
  // then runs again on the general path, these results dropped)
  uint32_t* ug_grid;
  uint32_t ug_t0, ug_step, ug_kk, ug_n;
  uint32_t ug_pieces;  // waves a span (0: wps_log2's blocks)
  // (the uniform path's speculative aligned group, launched before the host
  // has read the call state back) the kept-span count and the class keys from
  // the device; the group is attempted iff ug_spec_fits(); non-members write
  // nothing (there is no E yet)
  const uint64_t* spec_n_kept;
  const uint32_t* spec_go;  // Small.ug_go: ug_spec_fits() of the call state, set by the kept-list kernel
};


// bucket b's timestamp of the key's span (Span.java:399: the mean of its cells' ts)
DEVI uint32_t ug_bucket_ts(const FapArgs& f, uint32_t b) {
  const uint32_t sb = b * f.ug_kk, m = min(sb + f.ug_kk, f.ug_n) - sb;
  return f.ug_t0 + sb * f.ug_step + (uint32_t)((uint64_t)f.ug_step * (m - 1) / 2);
}

DEVI int64_t fap_neutral(int op) { return op == 1 ? INT64_MAX : (op == 2 ? INT64_MIN : 0); }

// Blocks of 4 waves; 1 << wps_log2 waves per span (a span's rows split into
// that many contiguous pieces), 4 >> wps_log2 spans per block. (FAP: one wave
// per span.) The body of k_ds_reg and of the uniform path's k_ug_ds_reg.
// (SPEC: the speculative aligned group, FapArgs.spec_*; a template argument,
// so the other launches carry none of its code)
template <int AGG, bool SPEC = false>
DEVI void ds_reg_body(const DecodeArgs& a, const SpanDsArgs& g, const uint32_t* ncells, const uint32_t* vlen,
                      uint32_t wps_log2, const FapArgs& fap) {
  __shared__ uint64_t s_v[4][DCH];
  __shared__ int64_t s_bk[4][WAVE];
  __shared__ int64_t s_part[WAVE];
  __shared__ uint32_t s_bad[4];
  const int lane = lane_id();
  const uint32_t wib = ufl(threadIdx.x / WAVE);  // (uniform: the span prologue and the row walk use scalar loads)
  // (the uniform path's E variant: ug_pieces waves a span, anywhere in the
  // grid — its pieces need no agreement, an outsider breaks the whole call)
  const uint32_t gw = blockIdx.x * 4u + wib;
  const uint32_t wps = fap.ug_pieces ? fap.ug_pieces : 1u << wps_log2;
  const uint32_t piece = fap.ug_pieces ? gw % wps : wib & (wps - 1);
  const uint32_t k = fap.ug_pieces ? gw / wps : blockIdx.x * (4u >> wps_log2) + (wib >> wps_log2);
  const int fop = fap.op;
  if (fop >= 0) {
    if (threadIdx.x < WAVE) s_part[threadIdx.x] = fap_neutral(fop);
    __syncthreads();
  }
  if (fap.ug_grid && blockIdx.x == 0) {
    const uint32_t nbk = (fap.ug_n + fap.ug_kk - 1) / fap.ug_kk;
    for (uint32_t b = threadIdx.x; b < nbk; b += blockDim.x) fap.ug_grid[b] = ug_bucket_ts(fap, b);
  }
  const int64_t I = a.interval;
  // (speculative: the kept count from the call state, the whole launch idle
  // unless the group is one)
  constexpr bool spec = SPEC;
  const uint32_t nk = spec ? (uint32_t)sld(fap.spec_n_kept) : a.n_kept;
  // (scalar loads and a wave-uniform verdict: a per-lane `ok` would turn the
  // span prologue's scalar loads and branches into vector ones)
  const bool go = !spec || sld(fap.spec_go) != 0;
  bool ok = go && k < nk && I > 0;
  uint32_t s = 0, W = 0, nb = 0;
  bool flt = false;
  RegSpan sp = {};
  uint64_t r0 = 0, r1 = 0, ra = 0, rb = 0;
  if (ok) {
    s = sld(&a.kept[k]);
    r0 = sld(&a.span_row_start[s]);
    r1 = sld(&a.span_row_start[s + 1]);
    sp.n = sld(&a.sp_ncells[s]);
    ok = sld(&a.sp_q1[s]) < 0 && sld(&a.sp_ovf_cell[s]) < 0 && sp.n > 0 && r1 > r0;
  }
  if (ok) {  // the first row: width, type, t0 and the cadence from its first two cells
    const uint32_t nc = sld(&ncells[r0]), vl = sld(&vlen[r0]);
    const uint32_t vb = nc > 1 ? vl - 1 : vl;
    W = nc != 0 && vb == (vb / nc) * nc ? vb / nc : 0;
    const uint64_t qo = sld(&a.row_qual_off[r0]);
    ok = (W == 8 || W == 4) && sld_u8(&a.row_ok[r0]) != 0 && (qo & 7) == 0 && (sp.n == 1 || nc >= 2);
    if (ok) {
      const uint32_t w = sld((const uint32_t*)(a.qual + qo));  // cells 0 and 1, big-endian
      const uint32_t q0 = ((w & 0xFF) << 8) | ((w >> 8) & 0xFF), q1 = ((w >> 16) & 0xFF) << 8 | (w >> 24);
      const uint32_t base = sld(&a.row_base[r0]);
      flt = (q0 & 8) != 0;
      sp.t0 = base + (q0 >> 4);
      const int64_t st = sp.n == 1 ? 1 : (int64_t)(base + (q1 >> 4)) - (int64_t)sp.t0;
      ok = st >= 1 && (int64_t)sp.t0 >= a.start &&
           (int64_t)sp.t0 + (int64_t)(sp.n - 1) * st <= 0xFFFFFFFFll;  // (no seek inside the span)
      sp.step = (uint32_t)st;
      sp.kk = (uint32_t)((I + st - 1) / st);
      sp.dkk.init(sp.kk);
      nb = (sp.n + sp.kk - 1) / sp.kk;
      sp.eo = sld(&a.e_off[k]);
      sp.cap = (uint32_t)sld(&a.sp_cap[s]);
      ok = ok && nb <= sp.cap;
    }
  }
  if (ok) {  // this wave's rows: a contiguous piece that starts at a bucket head
    const uint64_t rp = (r1 - r0 + wps - 1) / wps;
    ra = min(r0 + piece * rp, r1);
    rb = min(ra + rp, r1);
    if (ra < rb && piece > 0) ok = sld(&a.row_cell0[ra]) % sp.kk == 0;
    if (ok && ra < rb) ok = reg_rows_ok(a, sp, ra, rb, W);
  }
  // an aligned-group member: its buckets go to the block partial, not to E
  const bool fused = fop >= 0 && ok && !flt && nb <= WAVE;
  if (spec && !fused) ok = false;
  const int efop = fap.ug_grid ? -2 : -1;
  const int sfop = fused ? fop : efop;
  if (ok && ra < rb) {
    bool fail;
    if (W == 8)
      fail = flt ? reg_piece<AGG, 8, true>(a, sp, ra, rb, ncells, s_v[wib], s_bk[wib], efop, s_part)
                 : reg_piece<AGG, 8, false>(a, sp, ra, rb, ncells, s_v[wib], s_bk[wib], sfop, s_part);
    else
      fail = flt ? reg_piece<AGG, 4, true>(a, sp, ra, rb, ncells, s_v[wib], s_bk[wib], efop, s_part)
                 : reg_piece<AGG, 4, false>(a, sp, ra, rb, ncells, s_v[wib], s_bk[wib], sfop, s_part);
    ok = !fail;
  }
  if (wps > 1 && !fap.ug_pieces) {  // the span's pieces agree (every wave of the block reaches this)
    if (lane == 0) s_bad[wib] = ok ? 0u : 1u;
    __syncthreads();
    uint32_t any = 0;
    for (uint32_t i = 0; i < wps; i++) any |= s_bad[(wib & ~(wps - 1)) + i];
    ok = any == 0;
  }
  if (fop >= 0 && go && k < nk && lane == 0) {  // the group's class: one key, no span outside it
    if (!(ok && fused)) {
      if (!*(volatile uint32_t*)fap.broken) atomicOr(fap.broken, 1u);
    } else {
      const unsigned long long k1 = ((unsigned long long)sp.t0 << 32) | sp.n, k2 = sp.step;
      volatile unsigned long long* kv = fap.key;
      if (k1 < kv[0]) atomicMin(&fap.key[0], k1);
      if (k1 > kv[1]) atomicMax(&fap.key[1], k1);
      if (k2 < kv[2]) atomicMin(&fap.key[2], k2);
      if (k2 > kv[3]) atomicMax(&fap.key[3], k2);
    }
  }
  if (spec) {
    // (nothing past the class bookkeeping above: no list, no E)
  } else if (k < nk) {
    if (!ok && fap.ug_grid) {  // (a uniform group's outsider: see FapArgs.ug_grid)
      if (lane == 0 && !*(volatile uint32_t*)fap.broken) atomicOr(fap.broken, 1u);  // (any piece)
    } else if (!ok) {
      if (piece == 0 && lane == 0 && !fap.rewrite) {  // the whole span to k_ds_spans
        const uint32_t sg = blockIdx.x % g.nseg;
        g.list[(uint64_t)sg * g.seg_cap + atomicAdd(&g.list_count[sg], 1u)] = k;
      }
    } else if (!fap.rewrite) {
      if (piece == 0 && lane == 0) {
        a.e_len[k] = nb;
        a.e_bad[k] = -1;
        if (flt) {
          if (!a.gflags[0]) atomicOr(&a.gflags[0], 1u);
          if (!a.rate) {  // F*: the first bucket's ts + 1
            const int64_t fs = (int64_t)sp.t0 + (int64_t)((uint64_t)sp.step * (min(sp.kk, sp.n) - 1) / 2) + 1;
            if ((unsigned long long)fs > *(volatile unsigned long long*)a.fstar)
              atomicMax(a.fstar, (unsigned long long)fs);
          }
        } else if (!a.gflags[1]) {
          atomicOr(&a.gflags[1], 1u);
        }
      }
      if (g.bitmap) {  // G: the span's bucket timestamps <= end (rate: from the second)
        for (uint32_t b = piece * WAVE + lane; b < nb; b += WAVE * wps) {
          if (g.rate && b == 0) continue;
          const uint32_t sb = b * sp.kk, m = min(sb + sp.kk, sp.n) - sb;
          const int64_t t = (int64_t)sp.t0 + (int64_t)sb * sp.step + (int64_t)((uint64_t)sp.step * (m - 1) / 2);
          if (t > g.hi || t < g.lo) continue;
          const uint64_t off = (uint64_t)(t - g.lo);
          const uint32_t bit = 1u << (off & 31);
          uint32_t* w = &g.bitmap[off >> 5];
          if (!(*w & bit)) atomicOr(w, bit);
        }
      }
    }
  }
  if (fop >= 0) {  // the block's partial row
    __syncthreads();
    if (threadIdx.x < WAVE) {
      const int64_t v = s_part[threadIdx.x];
      if (!fap.copies) {
        fap.part[(uint64_t)blockIdx.x * WAVE + threadIdx.x] = v;
      } else if (v != fap_neutral(fop)) {
        unsigned long long* c = fap.copies + (uint64_t)(blockIdx.x % fap.ncopy) * WAVE + threadIdx.x;
        if (fop == 0) atomicAdd(c, (unsigned long long)v);
        else if (fop == 1) atomicMin((long long*)c, (long long)v);
        else atomicMax((long long*)c, (long long)v);
      }
    }
  }
}

#ifndef DS_WPE
#define DS_WPE 7  // waves per SIMD the register allocation aims at (C2, same box: the compiler's 83 VGPRs
                  // 0.165 ms, 7: 0.150, 8: 0.161)
#endif
template <int AGG>
__global__ void __launch_bounds__(256)
#if DS_WPE
__attribute__((amdgpu_waves_per_eu(DS_WPE, DS_WPE)))
#endif
k_ds_reg(DecodeArgs a, SpanDsArgs g, const uint32_t* ncells,
                                                const uint32_t* vlen, uint32_t wps_log2, FapArgs fap) {
  // (dynamic LDS: padding that caps the resident blocks per CU, see LaunchChunks)
  extern __shared__ uint8_t s_pad[];
  if (threadIdx.x == 0 && a.n_kept == 0xFFFFFFFFu) s_pad[0] = 1;
  ds_reg_body<AGG>(a, g, ncells, vlen, wps_log2, fap);
}

// FAP rows -> one 1-chunk partial per t: block b (16 waves) combines rows
// b * 16 + w + i * 16 gridDim.x (a wave per 512-B row, four rows in flight),
// then its waves in LDS, into tmp[b].
template <int OP>
DEVI int64_t fap_comb(int64_t x, int64_t y) {
  if (OP == 0) return ladd(x, y);
  if (OP == 1) return y < x ? y : x;
  return y > x ? y : x;
}
template <int OP>
DEVI int64_t fap_rows_wave(const int64_t* rows, uint32_t r, uint32_t stride, uint32_t nrows) {
  const int lane = lane_id();
  int64_t acc = fap_neutral(OP);
  // (8 rows in flight a wave: the single-block final reduce of ~250 rows is
  // a chain of round trips)
  for (; r + 7 * stride < nrows; r += 8 * stride) {
    int64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = rows[(uint64_t)(r + u * stride) * WAVE + lane];
#pragma unroll
    for (int u = 0; u < 8; u++) acc = fap_comb<OP>(acc, v[u]);
  }
  for (; r + 3 * stride < nrows; r += 4 * stride) {
    const int64_t v0 = rows[(uint64_t)r * WAVE + lane], v1 = rows[(uint64_t)(r + stride) * WAVE + lane];
    const int64_t v2 = rows[(uint64_t)(r + 2 * stride) * WAVE + lane], v3 = rows[(uint64_t)(r + 3 * stride) * WAVE + lane];
    acc = fap_comb<OP>(fap_comb<OP>(acc, v0), fap_comb<OP>(fap_comb<OP>(v1, v2), v3));
  }
  for (; r < nrows; r += stride) acc = fap_comb<OP>(acc, rows[(uint64_t)r * WAVE + lane]);
  return acc;
}
template <int OP>
DEVI int64_t fap_block_comb(int64_t acc, int64_t (*s)[WAVE]) {
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  s[w][lane] = acc;
  __syncthreads();
  if (w == 0)
    for (uint32_t i = 1; i < 16; i++) acc = fap_comb<OP>(acc, s[i][lane]);
  return acc;
}
template <int OP>
__global__ void __launch_bounds__(1024) k_fap_rows(const int64_t* part, uint32_t nrows, int64_t* tmp) {
  __shared__ int64_t s[16][WAVE];
  const uint32_t w = threadIdx.x / WAVE;
  int64_t acc = fap_rows_wave<OP>(part, blockIdx.x * 16 + w, gridDim.x * 16, nrows);
  acc = fap_block_comb<OP>(acc, s);
  if (w == 0) tmp[(uint64_t)blockIdx.x * WAVE + lane_id()] = acc;
}
// ... then the rows of tmp in one block; p_* as k_reduce's acc_store for a
// 1-chunk MODE_INT reduce: every kept span active at every t
template <int OP>
__global__ void __launch_bounds__(1024) k_fap_final(const int64_t* tmp, uint32_t n, uint64_t T, uint32_t n_kept,
                                                    int64_t* p_i, uint32_t* p_cnt, uint8_t* p_flag) {
  __shared__ int64_t s[16][WAVE];
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  int64_t acc = fap_rows_wave<OP>(tmp, w, 16, n);
  acc = fap_block_comb<OP>(acc, s);
  if (w == 0 && (uint64_t)lane < T) {
    p_i[lane] = acc;
    p_cnt[lane] = n_kept;
    p_flag[lane] = 0;
  }
}

// The same as 64 slots for an exchange (sharded optimistic finish): T read on
// the device, neutral slots past it.
template <int OP>
__global__ void __launch_bounds__(1024) k_fap_final64(const int64_t* tmp, uint32_t n, const uint64_t* Tp,
                                                      uint32_t n_kept, int64_t* p_i, uint32_t* p_cnt) {
  __shared__ int64_t s[16][WAVE];
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  int64_t acc = fap_rows_wave<OP>(tmp, w, 16, n);
  acc = fap_block_comb<OP>(acc, s);
  if (w == 0) {
    const bool in = (uint64_t)lane < *(volatile const uint64_t*)Tp;
    p_i[lane] = in ? acc : fap_neutral(OP);
    p_cnt[lane] = in ? n_kept : 0u;
  }
}

// The same, unsharded: the final values straight away (k_finalize_seq's
// finalize_one on the one-chunk accumulator), one launch instead of two.
template <int OP, int AGG>
__global__ void __launch_bounds__(1024) k_fap_final_out(const int64_t* tmp, uint32_t n, uint32_t n_kept,
                                                        FinalArgs f) {
  __shared__ int64_t s[16][WAVE];
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  int64_t acc = fap_rows_wave<OP>(tmp, w, 16, n);
  acc = fap_block_comb<OP>(acc, s);
  if (w == 0 && (uint64_t)lane < f.T) {
    Acc a;
    acc_init(a);
    a.cnt = n_kept;
    a.ia = acc;
    finalize_one<AGG, MODE_INT, false>(f, (uint64_t)lane, a);
  }
}

}  // namespace tsdb
