// batch.hip — tsdbhip_spangroup_run_batch: every SpanGroup of one query's
// GROUP BY (TsdbQuery.groupByAndAggregate, TsdbQuery.java:294-363) in one
// call. Included by api.hip after spangroup_run (unity build).
//
//   k_assemble ... k_kept_scatter   once over all spans (as spangroup_run)
//   k_group_stats                   kept range, aggregatedSize, bounds / group [sync 1]
//   k_decode_* / k_ds_spans         once over all kept spans (no grid marking) [sync 2]
//   k_group_summary                 E_EMPTY_SPAN, F*_g, int/float flags per group
//   k_grid_mark_seg .. k_group_rebase  segmented union grids (one bitmap per group,
//                                   concatenated; pad word per group)          [sync 3]
//   k_reduce_seg + k_finalize_seg   all groups of one reduce mode per launch (wave ->
//                                   group, tile group, span chunk)
//   k_bad_index_seg                 lazy error index per group                  [sync 4]
//
// Any error the reference raises at group construction (E_EMPTY_SPAN,
// E_CAPACITY, E_UNSORTED, E_UNSUPPORTED) makes the batch re-run its groups one
// by one through spangroup_run, so each group reports its own code exactly as
// a lone SpanGroup would; so does a set of group grids too large for one
// segmented bitmap (sparse groups over a very wide time range).


template <int AGG, int MODE, bool RATE>
static void launch_seg(Slot* ctx, const ReduceArgs& r0, const FinalArgs& f0, const SegReduce& sr,
                       uint64_t waves, const SegGroup* sg, const uint64_t* goff, uint32_t G, uint64_t T_all,
                       GroupDev* gd) {
  if (waves && r0.d_info)  // span chunks without E spans (k_reduce's DONLY instantiation)
    LAUNCH((k_reduce_seg<AGG, MODE, RATE, true>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       ctx->stream, r0, sr);
  if (waves)
    LAUNCH((k_reduce_seg<AGG, MODE, RATE, false>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       ctx->stream, r0, sr);
  if (T_all)
    LAUNCH((k_finalize_seg<AGG, MODE, RATE>), dim3(grid_for(T_all, 256)), dim3(256), 0, ctx->stream,
                       r0, f0, sg, goff, G, T_all, gd);
}

struct LaunchSeg {
  template <int AGG, typename... A>
  static void run(Slot* ctx, int mode, bool rate, A&&... a) {
    if (rate) return launch_seg<AGG, MODE_DBL, true>(ctx, a...);
    if (mode == MODE_INT) return launch_seg<AGG, MODE_INT, false>(ctx, a...);
    if (mode == MODE_DBL) return launch_seg<AGG, MODE_DBL, false>(ctx, a...);
    launch_seg<AGG, MODE_DUAL, false>(ctx, a...);
  }
};

template <typename T>
static T* upload(Slot* ctx, const char* name, const std::vector<T>& v) {
  T* d = scratch<T>(ctx, name, v.size());
  if (v.empty()) return d;
  void* h = host_buf(ctx, v.size() * sizeof(T));
  std::memcpy(h, v.data(), v.size() * sizeof(T));
  HIPCHK(hipMemcpyAsync(d, h, v.size() * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));  // host_buf is reused by the next call
  return d;
}

// One group through the single-group path, with the error mapping of the
// tsdbhip_spangroup_run wrapper (HIP/RCCL failures propagate).
static int run_group_alone(Slot* ctx, const tsdbhip_sg_desc* sub, tsdbhip_sg_out* out) {
  try {
    return spangroup_run(ctx, sub, out);
  } catch (Fail& f) {
    if (f.code == TSDBHIP_E_HIP || f.code == TSDBHIP_E_RCCL) throw;
    out->err_code = f.code;
    out->err_index = 0;
    hipStreamSynchronize(ctx->stream);
    return f.code;
  }
}

// Groups one by one over the already staged (device) inputs.
static int batch_one_by_one(Slot* ctx, const tsdbhip_sg_desc& dd, uint32_t G, const uint32_t* gss,
                            tsdbhip_sg_out* outs) {
  int first = TSDBHIP_OK;
  for (uint32_t g = 0; g < G; g++) {
    tsdbhip_sg_desc sub = dd;
    sub.span_row_start = dd.span_row_start + gss[g];
    sub.n_spans = gss[g + 1] - gss[g];
    const int rc = run_group_alone(ctx, &sub, &outs[g]);
    if (rc && !first) first = rc;
  }
  return first;
}

static int spangroup_run_batch(Slot* ctx, const tsdbhip_sg_desc* d, uint32_t G, const uint32_t* gss,
                               tsdbhip_sg_out* outs) {
  const bool dev = (d->flags & TSDBHIP_DESC_DEVICE) != 0;
  const bool exact = (d->flags & TSDBHIP_EXACT_ORDER) != 0;
  const uint32_t S = d->n_spans;
  const uint64_t R = d->n_rows;
  const bool rate = d->rate != 0;
  const int agg = d->agg;
  const int ds_agg = d->ds_agg;
  const int32_t interval = d->ds_interval > 0 ? d->ds_interval : 0;
  hipStream_t st = ctx->stream;
  tsdbhip_timing tm = {};
  ctx->hot_kernel = TSDBHIP_HOT_NONE;
  ctx->time_reduce = false;
  for (uint32_t g = 0; g < G; g++) {
    outs[g].n_out = 0;
    outs[g].n_input_points = 0;
    outs[g].err_code = 0;
    outs[g].err_index = -1;
  }

  // ---- inputs in HBM (the same staging as spangroup_run) ----
  tsdbhip_sg_desc dd = *d;  // device view of the inputs
  dd.flags |= TSDBHIP_DESC_DEVICE;
  dd.span_row_start = stage(ctx, "in_srs", d->span_row_start, (size_t)S + 1, dev);
  dd.row_base = stage(ctx, "in_base", d->row_base, R, dev);
  dd.row_ncells = stage(ctx, "in_ncells", d->row_ncells, R, dev);
  dd.row_qual_off = stage(ctx, "in_qoff", d->row_qual_off, R, dev);
  dd.row_val_off = stage(ctx, "in_voff", d->row_val_off, R, dev);
  dd.row_val_len = stage(ctx, "in_vlen", d->row_val_len, R, dev);
  dd.qual_bytes = stage(ctx, "in_qual", d->qual_bytes, d->qual_nbytes, dev, 16);
  dd.val_bytes = stage(ctx, "in_val", d->val_bytes, d->val_nbytes, dev, 16);
  const uint64_t* span_row_start = dd.span_row_start;
  const uint32_t* row_ncells = dd.row_ncells;
  const uint32_t* row_val_len = dd.row_val_len;

  struct Small {
    unsigned long long err;  // err_raise key, ERR_NONE: none
    uint32_t gflags[2];
    unsigned long long range[2];
    unsigned long long fstar;
    unsigned long long n_input;
    uint64_t n_kept;
    uint64_t e_total;
    uint64_t T;
    unsigned long long bound[2];
  };
  Small* sm = scratch<Small>(ctx, "b_small", 1);
  {
    Small init = {};
    init.err = ERR_NONE;
    init.range[0] = ~0ull;
    init.bound[0] = ~0ull;
    std::memcpy(ctx->host_small, &init, sizeof init);
    HIPCHK(hipMemcpyAsync(sm, ctx->host_small, sizeof init, hipMemcpyHostToDevice, st));
  }
  std::memset(ctx->ev_alias, 0xff, sizeof ctx->ev_alias);  // (markers only here)
  HIPCHK(hipEventRecord(ctx->ev[0], st));

  // ---- assemble (every span of every group) ----
  uint8_t* row_ok = scratch<uint8_t>(ctx, "row_ok", R);
  uint32_t* row_cell0 = scratch<uint32_t>(ctx, "row_cell0", R);
  uint32_t* sp_ncells = scratch<uint32_t>(ctx, "sp_ncells", S);
  int64_t* sp_first = scratch<int64_t>(ctx, "sp_first", S);
  int64_t* sp_last = scratch<int64_t>(ctx, "sp_last", S);
  uint8_t* sp_kept = scratch<uint8_t>(ctx, "sp_kept", S);
  uint64_t* sp_cap = scratch<uint64_t>(ctx, "sp_cap", S);
  int64_t* sp_q1 = scratch<int64_t>(ctx, "sp_q1", S);
  int32_t* sp_q1s = scratch<int32_t>(ctx, "sp_q1s", S);
  int64_t* sp_q1rs = scratch<int64_t>(ctx, "sp_q1rs", 2ull * S);
  int64_t* sp_ovf = scratch<int64_t>(ctx, "sp_ovf", S);
  if (S) {
    AssembleArgs a;
    a.span_row_start = span_row_start; a.row_base = dd.row_base; a.row_ncells = row_ncells;
    a.row_qual_off = dd.row_qual_off; a.row_val_len = row_val_len; a.qual = dd.qual_bytes;
    a.n_spans = S; a.start = d->start_time; a.end = d->end_time; a.interval = interval;
    a.row_ok = row_ok; a.row_cell0 = row_cell0; a.sp_ncells = sp_ncells; a.sp_first = sp_first;
    a.sp_last = sp_last; a.sp_kept = sp_kept; a.sp_cap = sp_cap; a.sp_q1 = sp_q1;
    a.sp_q1_shift = sp_q1s; a.sp_q1_rs = sp_q1rs; a.sp_ovf_cell = sp_ovf; a.err = &sm->err;
    a.span0 = 0;
    a.row_val_off = nullptr;
    a.u_key1 = a.u_key2 = a.u_vo = a.u_qo = nullptr;
    uint32_t* alist = scratch<uint32_t>(ctx, "asm_list", S);
    uint32_t* acount = scratch<uint32_t>(ctx, "asm_count", 1, true);
    LAUNCH(k_assemble_fast, dim3(grid_for(S, 256)), dim3(256), 0, st, a, alist, acount);
    LAUNCH(k_assemble, dim3(grid_for(S, 4, 4096)), dim3(256), 0, st, a, (const uint32_t*)alist,
                       (const uint32_t*)acount);
  }
  uint64_t* kflag = scratch<uint64_t>(ctx, "kflag", S);
  uint64_t* kidx = scratch<uint64_t>(ctx, "kidx", S);
  uint64_t* eoff_s = scratch<uint64_t>(ctx, "eoff_s", S);
  uint32_t* kept = scratch<uint32_t>(ctx, "kept", S);
  uint64_t* eoff = scratch<uint64_t>(ctx, "eoff", S);
  uint32_t* kgrp = scratch<uint32_t>(ctx, "b_kgrp", S);
  GroupStat* stat = scratch<GroupStat>(ctx, "b_stat", G);
  const uint32_t* gss_d = upload(ctx, "b_gss", std::vector<uint32_t>(gss, gss + G + 1));
  if (S) {
    LAUNCH(k_kept_flags, dim3(grid_for(S, 256)), dim3(256), 0, st, sp_kept, kflag, S);
    dscan_u64(ctx, kflag, kidx, S, &sm->n_kept, "k");
    dscan_u64(ctx, sp_cap, eoff_s, S, &sm->e_total, "e");
    LAUNCH(k_kept_scatter, dim3(grid_for(S, 256, 1024)), dim3(256), 0, st, sp_kept, kidx, eoff_s,
                       sp_ncells, S, kept, eoff, &sm->n_input, sp_first, sp_last, sm->bound);
  }
  Small h;
  readback(ctx, &h, sm, sizeof h);
  if (h.err != ERR_NONE) return batch_one_by_one(ctx, dd, G, gss, outs);
  const uint32_t n_kept = (uint32_t)h.n_kept;
  LAUNCH(k_group_stats, dim3(std::min<uint32_t>(std::max<uint32_t>(G, 1), 65536)), dim3(256), 0, st,
                     gss_d, G, S, n_kept, sp_kept, kidx, sp_ncells, sp_first, sp_last, kgrp, stat);
  std::vector<GroupStat> gs(G);
  {
    void* hb = host_buf(ctx, sizeof(GroupStat) * std::max<uint32_t>(G, 1));
    HIPCHK(hipMemcpyAsync(hb, stat, sizeof(GroupStat) * G, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));  // sync 1
    std::memcpy(gs.data(), hb, sizeof(GroupStat) * G);
  }

  // ---- segmented bitmap geometry: group g over [max(start, first_g), min(end, last_g)]
  std::vector<int64_t> glo(G), ghi(G);
  std::vector<uint64_t> gwb(G);
  std::vector<uint32_t> gnw(G);
  uint64_t W = 0;
  for (uint32_t g = 0; g < G; g++) {
    int64_t lo = 1, hi = 0;
    if (gs[g].nk) {
      lo = std::max<int64_t>(d->start_time, gs[g].first);
      hi = std::min<int64_t>(d->end_time, gs[g].last);
    }
    glo[g] = lo;
    ghi[g] = hi;
    gnw[g] = lo <= hi ? (uint32_t)((uint64_t)(hi - lo + 1 + 31) / 32) : 0;
    gwb[g] = W;
    W += (uint64_t)gnw[g] + 1;
  }
  // ranks are u32 and the bitmaps live in HBM: very sparse wide-range groups
  // go one by one (each reuses a single bitmap)
  if (W * 32 >= (1ull << 32) || W > (1ull << 28)) return batch_one_by_one(ctx, dd, G, gss, outs);
  GroupGrid q;
  q.lo = upload(ctx, "b_lo", glo);
  q.hi = upload(ctx, "b_hi", ghi);
  q.wbase = upload(ctx, "b_wbase", gwb);
  q.nw = upload(ctx, "b_nw", gnw);
  uint32_t* wgrp = scratch<uint32_t>(ctx, "b_wgrp", W);
  q.wgrp = wgrp;

  // ---- decode (+ downsample), every kept span ----
  const uint64_t e_total = h.e_total;
  uint32_t* e_ts = scratch<uint32_t>(ctx, "e_ts", e_total);
  int64_t* e_val = scratch<int64_t>(ctx, "e_val", e_total);
  uint8_t* e_flt = scratch<uint8_t>(ctx, "e_flt", e_total);
  uint32_t* e_len = scratch<uint32_t>(ctx, "e_len", n_kept);
  int64_t* e_bad = scratch<int64_t>(ctx, "e_bad", n_kept);
  DecodeArgs da;
  da.span_row_start = span_row_start; da.row_base = dd.row_base; da.row_qual_off = dd.row_qual_off;
  da.row_val_off = dd.row_val_off; da.qual = dd.qual_bytes; da.val = dd.val_bytes; da.row_ok = row_ok;
  da.row_cell0 = row_cell0; da.kept = kept; da.n_kept = n_kept; da.sp_ncells = sp_ncells; da.sp_q1 = sp_q1;
  da.sp_q1_shift = sp_q1s; da.sp_q1_rs = sp_q1rs; da.sp_ovf_cell = sp_ovf; da.sp_cap = sp_cap; da.e_off = eoff; da.e_ts = e_ts;
  da.e_val = e_val; da.e_flt = e_flt; da.e_len = e_len; da.e_bad = e_bad; da.start = d->start_time;
  da.end = d->end_time; da.interval = interval; da.ds_agg = ds_agg; da.rate = rate; da.err = &sm->err;
  da.gflags = sm->gflags; da.range = sm->range; da.fstar = &sm->fstar; da.span0 = 0; da.sp_first = sp_first;
  da.row_ncells = dd.row_ncells; da.row_val_len = dd.row_val_len;
  HIPCHK(hipEventRecord(ctx->ev[1], st));
  bool direct = false;  // k_direct_scan took the no-downsampling path
  DirectArgs dg = {};
  if (n_kept) {
    const unsigned blocks = grid_for(n_kept, 4, 65536);
    const bool no_direct = ctx->opt.decode == DEC_FAST;  // (tests: the E path for every span)
    const bool fast = R > 0 && h.n_input / R >= 64;  // wide (hourly compacted) rows
    da.fb_list = scratch<uint32_t>(ctx, "fb_list", n_kept);
    da.fb_count = scratch<uint32_t>(ctx, "fb_count", 1, true);
    da.use_fb = 0;
    da.span_list = nullptr;
    da.span_count = nullptr;
    DecodeArgs ga = da;
    ga.use_fb = 1;
    ctx->hot_kernel = fast ? TSDBHIP_HOT_DECODE_FAST : TSDBHIP_HOT_DECODE_GEN;
    HIPCHK(hipEventRecord(ctx->ev[8], st));
    if (!fast) {
      if (interval == 0) LAUNCH(k_decode_nods, dim3(blocks), dim3(256), 0, st, da);
      else launch_agg<LaunchGeneralDs>(ds_agg, ctx, blocks, da);
      HIPCHK(hipEventRecord(ctx->ev[9], st));
    } else if (interval == 0) {
      DecodeArgs fa = da;
      direct = !no_direct;
      if (direct) {
        // regular-cadence spans on consecutive grid ranks of their group skip E
        // (k_direct.hip); the scan only proves the cadence here, the group
        // grids are marked after decode (k_direct_mark_seg)
        dg.info = scratch<uint32_t>(ctx, "d_info", n_kept);
        dg.n = scratch<uint32_t>(ctx, "d_n", n_kept);
        dg.x0 = scratch<uint32_t>(ctx, "d_x0", n_kept);
        dg.step = scratch<uint32_t>(ctx, "d_step", n_kept);
        dg.voff = scratch<uint64_t>(ctx, "d_voff", n_kept);
        dg.c0 = scratch<uint32_t>(ctx, "d_c0", n_kept);
        dg.r0 = scratch<uint64_t>(ctx, "d_r0", n_kept);
        dg.ga = scratch<uint32_t>(ctx, "d_ga", n_kept);
        dg.row_cpre = scratch<uint32_t>(ctx, "row_cpre", R);
        dg.list = scratch<uint32_t>(ctx, "d_list", n_kept);
        dg.list_count = scratch<uint32_t>(ctx, "d_list_count", 1, true);
        dg.bitmap = nullptr;
        dg.lo = 0;
        dg.hi = -1;
        dg.rate = rate;
        ctx->hot_kernel = TSDBHIP_HOT_REDUCE_DIRECT;  // timed around the reduce launches
        // (spans per wave: 32 for big groups; fewer below ~64k spans, so a
        // small group still spreads over ~2048 waves instead of a handful)
        dg.batch = std::max<uint32_t>(1, std::min<uint32_t>(DIRB, n_kept / 2048));
        LAUNCH(k_direct_scan, dim3(grid_for(n_kept, 4 * dg.batch, 1u << 20)), dim3(256), 0, st, da, dg,
                           row_ncells, row_val_len);
        fa.span_list = dg.list;
        fa.span_count = dg.list_count;
      }
      const unsigned lblocks = fa.span_list ? std::min(blocks, 1024u) : blocks;
      LAUNCH((k_decode_fast<0, false>), dim3(lblocks), dim3(256), 0, st, fa, row_ncells, row_val_len);
      if (!direct) HIPCHK(hipEventRecord(ctx->ev[9], st));
      LAUNCH(k_decode_nods, dim3(std::min(blocks, 1024u)), dim3(256), 0, st, ga);
    } else {
      DecodeArgs fa = da;
      if (ds_agg != 4) {
        SpanDsArgs sg = {};
        sg.bitmap = nullptr;  // group grids are marked after decode
        sg.rate = rate;
        launch_agg<LaunchChunks>(ds_agg, ctx, da, fa, row_ncells, row_val_len, sg, R);
      }
      const unsigned lblocks = fa.span_list ? std::min(blocks, 1024u) : blocks;
      launch_agg<LaunchFastDs>(ds_agg, ctx, lblocks, fa, row_ncells, row_val_len);
      if (ctx->hot_kernel == TSDBHIP_HOT_DECODE_FAST) HIPCHK(hipEventRecord(ctx->ev[9], st));
      launch_agg<LaunchGeneralDs>(ds_agg, ctx, std::min(blocks, 1024u), ga);
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  readback(ctx, &h, sm, sizeof h);  // sync 2: decode errors, global int/float flags
  if (h.err != ERR_NONE) return batch_one_by_one(ctx, dd, G, gss, outs);
  const bool anyf = h.gflags[0] != 0, anyi = h.gflags[1] != 0;

  // ---- per-group summary and segmented union grids ----
  GroupDev* gd = scratch<GroupDev>(ctx, "b_gd", G);
  LAUNCH(k_group_init, dim3(grid_for(G, 256)), dim3(256), 0, st, gd, G);
  HIPCHK(hipEventRecord(ctx->ev[3], st));
  const uint32_t* d_info = direct ? dg.info : nullptr;
  uint32_t* bitmap = scratch<uint32_t>(ctx, "bitmap", W, true);
  uint32_t* word_rank = scratch<uint32_t>(ctx, "word_rank", W);
  const uint64_t nb = (W + 1023) / 1024;
  uint32_t* bsum = scratch<uint32_t>(ctx, "grid_bsum", nb);
  LAUNCH(k_group_words, dim3(std::min<uint32_t>(std::max<uint32_t>(G, 1), 65536)), dim3(256), 0, st, q,
                     G, wgrp);
  if (n_kept)
    LAUNCH(k_grid_mark_seg, dim3(grid_for(n_kept, 4, 65536)), dim3(256), 0, st, eoff, e_len, e_ts,
                       n_kept, (int32_t)rate, kgrp, q, bitmap, d_info);
  if (direct && n_kept)
    LAUNCH(k_direct_mark_seg, dim3(grid_for(n_kept, 4 * WAVE, 16384)), dim3(256), 0, st, dg, n_kept,
                       kgrp, q, bitmap);
  GridArgs ga = {};
  std::memset(&ga, 0, sizeof ga);
  ga.bitmap = bitmap; ga.nwords = W; ga.word_rank = word_rank; ga.block_sum = bsum; ga.total = &sm->T;
  LAUNCH(k_grid_popc, dim3((unsigned)nb), dim3(256), 0, st, ga);
  if (nb > 1) LAUNCH(k_grid_scan_blocks, dim3(1), dim3(256), 0, st, ga, (uint32_t)nb);
  readback(ctx, &h, sm, sizeof h);  // total |G| over the groups (grid buffer size)
  const uint64_t T_all = h.T;
  uint32_t* gridv = scratch<uint32_t>(ctx, "grid", T_all);
  LAUNCH(k_grid_emit_seg, dim3(grid_for(W, 256)), dim3(256), 0, st, bitmap, word_rank,
                     (const uint32_t*)bsum, W, q, gridv);
  LAUNCH(k_group_T, dim3(grid_for(G, 256)), dim3(256), 0, st, q, G, (const uint32_t*)word_rank, gd);
  LAUNCH(k_group_rebase, dim3(grid_for(W, 256)), dim3(256), 0, st, q, W, (const GroupDev*)gd,
                     word_rank);
  if (direct && n_kept) {
    // candidates whose points are not consecutive ranks of their group grid
    // need E (their grid points are already marked)
    HIPCHK(hipMemsetAsync(dg.list_count, 0, 4, st));
    HIPCHK(hipMemsetAsync(da.fb_count, 0, 4, st));
    LAUNCH(k_direct_verify_seg, dim3(grid_for(n_kept, 256)), dim3(256), 0, st, dg, n_kept, kgrp, q,
                       (const uint32_t*)bitmap, (const uint32_t*)word_rank);
    DecodeArgs fa = da;
    fa.span_list = dg.list;
    fa.span_count = dg.list_count;
    const unsigned vb = std::min(grid_for(n_kept, 4, 65536), 1024u);
    LAUNCH((k_decode_fast<0, false>), dim3(vb), dim3(256), 0, st, fa, row_ncells, row_val_len);
    DecodeArgs gfa = da;
    gfa.use_fb = 1;
    LAUNCH(k_decode_nods, dim3(vb), dim3(256), 0, st, gfa);
  }
  // E_EMPTY_SPAN, F*_g and the group's int/float flags, over final E / direct spans
  if (n_kept)
    LAUNCH(k_group_summary, dim3(grid_for(n_kept, 4, 65536)), dim3(256), 0, st, eoff, e_len, e_ts,
                       e_flt, n_kept, (int32_t)rate, (int32_t)(!rate && anyf && anyi), kgrp, d_info,
                       (const uint32_t*)dg.x0, gd, &sm->err);
  HIPCHK(hipEventRecord(ctx->ev[4], st));
  std::vector<GroupDev> gh(G);
  auto read_groups = [&]() {
    void* hb = host_buf(ctx, sizeof(GroupDev) * std::max<uint32_t>(G, 1));
    HIPCHK(hipMemcpyAsync(hb, gd, sizeof(GroupDev) * G, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(gh.data(), hb, sizeof(GroupDev) * G);
  };
  read_groups();  // sync 3
  readback(ctx, &h, sm, sizeof h);
  if (h.err != ERR_NONE) return batch_one_by_one(ctx, dd, G, gss, outs);
  tm.n_grid = T_all;

  // ---- reduce: one k_reduce_seg + k_finalize_seg per reduce mode present,
  // each wave mapped to (group, tile group, span chunk) ----
  int64_t* out_ts = scratch<int64_t>(ctx, "out_ts", T_all);
  uint8_t* out_isint = scratch<uint8_t>(ctx, "out_isint", T_all);
  int64_t* out_bits = scratch<int64_t>(ctx, "out_bits", T_all);
  auto mode_of = [&](uint32_t g) {
    if (rate) return (int)MODE_DBL;
    const bool f = anyf && anyi ? (gh[g].gfl & 1u) != 0 : anyf;
    const bool i = anyf && anyi ? (gh[g].gfl & 2u) != 0 : anyi;
    return !f ? (int)MODE_INT : (!i ? (int)MODE_DBL : (int)MODE_DUAL);
  };
  std::vector<SegGroup> sgv(G);
  std::vector<uint64_t> goffv(G);
  std::vector<uint32_t> glist[3];
  std::vector<uint64_t> wstart[3];
  for (auto& w : wstart) w.push_back(0);
  uint64_t poff = 0, coff = 0, choff = 0;
  std::vector<uint64_t> choffv(G, 0);
  for (uint32_t g = 0; g < G; g++) {
    SegGroup& x = sgv[g];
    std::memset(&x, 0, sizeof x);
    x.k0 = gs[g].k0;
    x.nk = (uint32_t)gs[g].nk;
    x.goff = gh[g].goff;
    x.T = gh[g].T;
    x.wbase = gwb[g];
    x.lo = glo[g];
    x.fstar = gh[g].fstar;
    x.mode = (uint32_t)mode_of(g);
    goffv[g] = x.goff;
    if (!x.T) continue;
    // the batch shares the single-group wave budget in proportion to spans
    const double share = n_kept ? (double)x.nk / n_kept : 1.0;
    // integer dev in one span-ordered pass: the reference's sequential
    // Welford, bit-exact after the (long) truncation (Aggregators.java:196-217)
    const bool seq = exact || (agg == TSDBHIP_AGG_DEV && x.mode != MODE_DBL);
    const ReduceGeom rg = reduce_geom(x.T, x.nk, seq, std::max<uint64_t>(64, (uint64_t)(16384 * share)),
                                      std::max<uint64_t>(16, (uint64_t)(2048 * share)));
    x.spc = rg.spc; x.n_chunks = rg.n_chunks; x.tpw = rg.tpw; x.ntg = rg.ntg;
    x.poff = poff;
    poff += (uint64_t)rg.n_chunks * x.T;
    x.coff = coff;
    coff += rg.n_waves * rg.spc;
    x.choff = choff;
    choffv[g] = choff;
    choff += rg.n_chunks;
    glist[x.mode].push_back(g);
    wstart[x.mode].push_back(wstart[x.mode].back() + rg.n_waves);
  }
  ReduceArgs r0;
  std::memset(&r0, 0, sizeof r0);
  r0.e_off = eoff; r0.e_len = e_len; r0.e_ts = e_ts; r0.e_val = e_val; r0.e_flt = e_flt; r0.kept = kept;
  r0.grid = gridv; r0.bitmap = bitmap; r0.word_rank = word_rank; r0.exact = exact ? 1 : 0;
  auto alloc_reduce = [&](ReduceArgs& r, uint64_t ncur, uint64_t npart) {
    r.ptr = scratch<uint32_t>(ctx, "cursor", ncur);
    r.st_x = scratch<uint2>(ctx, "st_x", ncur);
    r.st_y = scratch<longlong2>(ctx, "st_y", ncur);
    r.st_rv = scratch<double>(ctx, "st_rv", ncur);
    r.st_f = scratch<uint32_t>(ctx, "st_f", ncur);
    r.p_cnt = scratch<uint32_t>(ctx, "p_cnt", npart);
    r.p_flag = scratch<uint8_t>(ctx, "p_flag", npart);
    r.p_i = scratch<int64_t>(ctx, "p_i", npart);
    r.p_d = scratch<double>(ctx, "p_d", npart);
    r.p_dhas = scratch<uint32_t>(ctx, "p_dhas", npart);
    if (agg == TSDBHIP_AGG_DEV) {
      r.p_wim = scratch<double>(ctx, "p_wim", npart);
      r.p_wiv = scratch<double>(ctx, "p_wiv", npart);
      r.p_wdm = scratch<double>(ctx, "p_wdm", npart);
      r.p_wdv = scratch<double>(ctx, "p_wdv", npart);
    }
  };
  alloc_reduce(r0, std::max<uint64_t>(coff, 1), std::max<uint64_t>(poff, 1));
  FinalArgs f0;
  std::memset(&f0, 0, sizeof f0);
  f0.grid = gridv; f0.rate = rate; f0.out_ts = out_ts; f0.out_isint = out_isint; f0.out_bits = out_bits;
  const SegGroup* sg_d = upload(ctx, "b_seg", sgv);
  const uint64_t* goff_d = upload(ctx, "b_goff", goffv);
  if (direct) {
    r0.d_info = dg.info; r0.d_n = dg.n; r0.d_ga = dg.ga; r0.d_voff = dg.voff; r0.d_x0 = dg.x0;
    r0.d_step = dg.step; r0.d_c0 = dg.c0; r0.d_r0 = dg.r0; r0.row_cpre = dg.row_cpre;
    r0.span_row_start = span_row_start; r0.row_ncells = row_ncells; r0.row_val_off = dd.row_val_off;
    r0.val = dd.val_bytes;
    uint32_t* ce = scratch<uint32_t>(ctx, "chunk_e", std::max<uint64_t>(choff, 1), true);
    const uint64_t* choff_d = upload(ctx, "b_choff", choffv);
    if (n_kept)
      LAUNCH(k_chunk_flags_seg, dim3(grid_for(n_kept, 256)), dim3(256), 0, st, (const uint32_t*)dg.info,
                         n_kept, (const uint32_t*)kgrp, sg_d, choff_d, ce);
    r0.chunk_e = ce;
    HIPCHK(hipEventRecord(ctx->ev[8], st));
  }
  for (int m = 0; m < 3; m++) {
    if (glist[m].empty()) continue;
    SegReduce sr;
    sr.sg = sg_d;
    sr.glist = upload(ctx, m == 0 ? "b_gl0" : m == 1 ? "b_gl1" : "b_gl2", glist[m]);
    sr.wv_start = upload(ctx, m == 0 ? "b_ws0" : m == 1 ? "b_ws1" : "b_ws2", wstart[m]);
    sr.n = (uint32_t)glist[m].size();
    launch_agg<LaunchSeg>(agg, ctx, m, rate, r0, f0, sr, wstart[m].back(), sg_d, goff_d, G, T_all, gd);
  }
  if (direct) HIPCHK(hipEventRecord(ctx->ev[9], st));  // (finalize included: small next to the reduce)
  if (n_kept)
    LAUNCH(k_bad_index_seg, dim3(grid_for(n_kept, 256)), dim3(256), 0, st, e_bad, eoff, e_ts, n_kept,
                       (int32_t)rate, kgrp, q, bitmap, word_rank, gd);
  HIPCHK(hipEventRecord(ctx->ev[5], st));
  read_groups();  // sync 4
  HIPCHK(hipStreamSynchronize(st));
  tm.decode_ms = ev_ms(ctx, 1, 2);
  if (ctx->hot_kernel) tm.hot_ms = ev_ms(ctx, 8, 9);
  tm.hot_kernel = ctx->hot_kernel;
  tm.grid_ms = ev_ms(ctx, 3, 4);
  tm.reduce_ms = ev_ms(ctx, 4, 5);
  tm.total_ms = ev_ms(ctx, 0, 5);
  tm.n_emitted = e_total;
  ctx->timing = tm;

  // ---- outputs: one D2H of the concatenated results, then per group ----
  const size_t ob = (size_t)T_all * 17;
  uint8_t* hb = (uint8_t*)host_buf(ctx, std::max<size_t>(ob, 64));
  int64_t* h_ts = (int64_t*)hb;
  int64_t* h_bits = (int64_t*)(hb + (size_t)T_all * 8);
  uint8_t* h_isint = hb + (size_t)T_all * 16;
  if (T_all) {
    HIPCHK(hipMemcpyAsync(h_ts, out_ts, T_all * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h_bits, out_bits, T_all * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h_isint, out_isint, T_all, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  int first = TSDBHIP_OK;
  for (uint32_t g = 0; g < G; g++) {
    tsdbhip_sg_out* o = &outs[g];
    o->n_input_points = gs[g].n_input;
    uint64_t n_ok = gh[g].T;
    int code = TSDBHIP_OK;
    int64_t err_at = -1;
    if (gh[g].bad_at != ~0ull) {
      err_at = (int64_t)(gh[g].bad_at >> 4);
      code = (gh[g].bad_at & 15) == BAD_OOB ? TSDBHIP_E_OUT_OF_BOUNDS : TSDBHIP_E_ILLEGAL_DATA;
    }
    if (gh[g].nan_t != ~0ull && (err_at < 0 || (int64_t)gh[g].nan_t < err_at)) {
      err_at = (int64_t)gh[g].nan_t;
      code = TSDBHIP_E_NAN_INF;
    }
    if (err_at >= 0) n_ok = (uint64_t)err_at;
    if (n_ok > o->capacity) {
      code = TSDBHIP_E_CAPACITY;
      n_ok = 0;
      err_at = -1;
    }
    const uint64_t go = gh[g].goff;
    if (n_ok) {
      std::memcpy(o->ts, h_ts + go, n_ok * 8);
      std::memcpy(o->bits, h_bits + go, n_ok * 8);
      std::memcpy(o->is_int, h_isint + go, n_ok);
    }
    o->n_out = n_ok;
    o->err_code = code;
    o->err_index = err_at;
    if (code && !first) first = code;
  }
  return first;
}

extern "C" int tsdbhip_spangroup_run_batch(tsdbhip_ctx* c, const tsdbhip_sg_desc* desc, uint32_t n_groups,
                                           const uint32_t* group_span_start, tsdbhip_sg_out* outs) {
  if (!c || !desc || !outs || !group_span_start || n_groups == 0) return TSDBHIP_E_INVALID_ARG;
  if (desc->agg > 4 || (desc->ds_interval > 0 && desc->ds_agg > 4) || desc->ds_interval < 0 ||
      desc->start_time < 0 || desc->end_time < 0 || (desc->flags & TSDBHIP_SHARDED) ||
      group_span_start[0] != 0 || group_span_start[n_groups] != desc->n_spans) {
    set_error(c, "invalid SpanGroup batch arguments");
    return TSDBHIP_E_INVALID_ARG;
  }
  for (uint32_t g = 0; g < n_groups; g++)
    if (group_span_start[g + 1] < group_span_start[g]) {
      set_error(c, "group_span_start not non-decreasing at group %u", g);
      return TSDBHIP_E_INVALID_ARG;
    }
  try {
    Lease L(plain_of(c));
    Slot* ctx = L.s;
    try {
      const int rc = spangroup_run_batch(ctx, desc, n_groups, group_span_start, outs);
      if (rc) set_error(ctx, "spangroup_run_batch: first failing group error %d", rc);
      return rc;
    } catch (Fail& f) {
      for (uint32_t g = 0; g < n_groups; g++) outs[g].err_code = f.code;
      set_error(ctx, "spangroup_run_batch: error %d", f.code);
      hipStreamSynchronize(ctx->stream);
      return f.code;
    }
  } catch (Fail& f) {
    for (uint32_t g = 0; g < n_groups; g++) outs[g].err_code = f.code;
    return f.code;
  }
}
