// Host side of the C-ABI (include/pinot_amd.h): segment residency, query planning (CNF filter, column
// slots, staging, accumulator layout, strategy) and result fetch. No CPU fallback: every query runs the
// HIP kernels; errors surface as negative return codes + pa_last_error().
#include "pa_host.h"

extern "C" {

pa_query* pa_query_create(const pa_query_spec* spec, int32_t num_segments) {
  if (!spec || num_segments < 0) {
    fail(PA_EINVAL, "bad query spec");
    return nullptr;
  }
  if (spec->num_leaves < 0 || spec->num_leaves > PA_MAX_LEAVES || spec->num_ops < 0 || spec->num_ops > PA_MAX_OPS ||
      spec->num_group_by < 0 || spec->num_group_by > PA_MAX_GROUP_BY || spec->num_aggs < 0 ||
      spec->num_aggs > PA_MAX_AGGS) {
    fail(PA_EINVAL, "query spec counts out of range");
    return nullptr;
  }
  pa_query* q = new pa_query();
  q->spec = *spec;
  q->nseg = num_segments;
  q->segs.assign(num_segments, nullptr);
  q->leaf_params.resize(num_segments);
  q->luts.resize(num_segments);
  q->remaps.resize(num_segments);
  q->has_remap.resize(num_segments);
  q->vremaps.assign(num_segments, std::vector<std::vector<int32_t>>(spec->num_aggs));
  return q;
}

int pa_query_bind_segment(pa_query* q, int32_t index, const pa_segment* seg, const pa_leaf_params* leaf_params,
                          const int32_t* const* group_remaps) {
  if (!q || !seg || index < 0 || index >= q->nseg) return fail(PA_EINVAL, "bad bind arguments");
  if (q->prepared) return fail(PA_EINVAL, "query already prepared");
  const pa_query_spec& s = q->spec;
  q->segs[index] = seg;
  q->leaf_params[index].assign(leaf_params, leaf_params + s.num_leaves);
  q->luts[index].assign(s.num_leaves, {});
  for (int l = 0; l < s.num_leaves; ++l) {
    const int kind = s.leaves[l].kind;
    if (kind == PA_LEAF_DICT_SET || kind == PA_LEAF_MV_DICT_SET) {
      auto it = seg->cols.find(s.leaves[l].column_id);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "leaf column missing in segment");
      if (!leaf_params[l].lut) return fail(PA_EINVAL, "DICT_SET leaf without lut");
      const size_t words = ((size_t)it->second->cardinality + 31) / 32;
      q->luts[index][l].assign(leaf_params[l].lut, leaf_params[l].lut + words);
    } else if (kind == PA_LEAF_RAW_SET) {  // (the values, 8 bytes each, kept as word pairs)
      auto it = seg->cols.find(s.leaves[l].column_id);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "leaf column missing in segment");
      const int64_t n = leaf_params[l].num_values;
      if (n < 0 || n > (int64_t(1) << 30) || (n > 0 && !leaf_params[l].values))
        return fail(PA_EINVAL, "RAW_SET leaf: bad value list");
      const bool integral = it->second->vtype == PA_INT || it->second->vtype == PA_LONG;
      const int64_t* vi = (const int64_t*)leaf_params[l].values;
      const double* vd = (const double*)leaf_params[l].values;
      for (int64_t i = 1; i < n; ++i)
        if (integral ? !(vi[i - 1] < vi[i]) : !(vd[i - 1] < vd[i]))
          return fail(PA_EINVAL, "RAW_SET leaf: values must be strictly ascending");
      const uint32_t* w = (const uint32_t*)leaf_params[l].values;
      q->luts[index][l].assign(w, w + 2 * n);
    }
  }
  q->remaps[index].assign(s.num_group_by, {});
  q->has_remap[index].assign(s.num_group_by, 0);
  for (int j = 0; j < s.num_group_by; ++j) {
    if (group_remaps && group_remaps[j]) {
      auto it = seg->cols.find(s.group_by_columns[j]);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "group-by column missing in segment");
      const int32_t card = it->second->cardinality;
      q->remaps[index][j].assign(group_remaps[j], group_remaps[j] + card);
      for (int32_t v : q->remaps[index][j])
        if (v < 0 || v >= s.group_by_cardinality[j]) return fail(PA_EINVAL, "group remap id outside the key space");
      q->has_remap[index][j] = 1;
    }
  }
  return PA_OK;
}

int pa_query_bind_value_remap(pa_query* q, int32_t index, int32_t agg, const int32_t* remap) {
  if (!q || index < 0 || index >= q->nseg || agg < 0 || agg >= q->spec.num_aggs) return fail(PA_EINVAL, "bad remap arguments");
  if (q->prepared) return fail(PA_EINVAL, "query already prepared");
  if (!q->segs[index]) return fail(PA_EINVAL, "bind the segment before its value remaps");
  const pa_agg_spec& A = q->spec.aggs[agg];
  if (A.type != PA_AGG_DISTINCTCOUNT) return fail(PA_EINVAL, "value remaps belong to DISTINCTCOUNT aggregations");
  auto it = q->segs[index]->cols.find(A.column_id);
  if (it == q->segs[index]->cols.end()) return fail(PA_EINVAL, "aggregation column missing in segment");
  q->vremaps[index][agg].clear();
  if (!remap) return PA_OK;
  const int32_t card = it->second->cardinality;
  q->vremaps[index][agg].assign(remap, remap + card);
  for (int32_t v : q->vremaps[index][agg])
    if (v < 0 || v >= A.num_values) return fail(PA_EINVAL, "value remap id outside the table-wide value dictionary");
  return PA_OK;
}

int pa_query_prepare(pa_query* q) {
  if (!q) return fail(PA_EINVAL, "null query");
  if (q->prepared) return PA_OK;
  for (int i = 0; i < q->nseg; ++i)
    if (!q->segs[i]) return fail(PA_EINVAL, "segment " + std::to_string(i) + " not bound");
  Prep P;
  std::memset(&q->hq, 0, sizeof(q->hq));
  int rc = plan_filter(q, P);
  if (!rc) rc = plan_slots(q, P);
  if (!rc) rc = plan_key_space(q, P);
  if (!rc) rc = plan_limit(q, P);
  if (!rc) rc = plan_gdense(q, P);
  if (!rc) rc = build_segments(q, P);
  if (!rc) rc = plan_walk(q, P);
  if (!rc) rc = plan_accumulators(q, P);
  TilePlan plan, count_plan;
  if (!rc) rc = plan_kernels(q, P, plan, count_plan);
  if (rc) return rc;

  // layout: tiles per segment, LDS regions (the count pass has its own staging), staged bytes
  void* dummy = nullptr;  // 256 readable bytes: source of the DMA padding instructions
  {
    std::vector<char> z(256, 0);
    rc = upload_owned(q, z.data(), z.size(), &dummy);
    if (rc) return rc;
  }
  const int nslots = (int)q->slot_cols.size();
  int64_t total_tiles = 0;
  apply_layout(q->hsegs, plan.steps, nslots, (int)q->literals.size(), dummy, &q->staged_bytes, &total_tiles);
  q->num_tiles = (uint64_t)total_tiles;
  q->lane_major = P.lm ? 1 : 0;
  q->dense_packed = P.gd_packed ? 1 : 0;
  q->plan_ring = plan.ring;
  q->plan_wg = plan.wg_per_cu;
  fill_devquery(q, P, plan, total_tiles);
  rc = plan_leaps(q, P);
  if (rc) return rc;

  // grid: persistent waves, enough workgroups to cover the CUs several times over
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
  }
  const int wg_cu = q->split_emit ? std::min(plan.wg_per_cu, q->emit_h_wg) : plan.wg_per_cu;
  const int64_t max_wg = (int64_t)cus * std::max(1, wg_cu);
  const int wpw = q->partitioned ? scan_waves(q->emit_strat) : scan_waves(q->strategy);
  const int64_t want = (total_tiles + wpw - 1) / wpw;
  q->grid = (int)std::max<int64_t>(1, std::min(max_wg, want));

  if (q->partitioned) {
    // the count pass: the same tiles, waves and grid; only the group-by and filter columns staged
    int64_t ct = 0;
    apply_layout(q->hsegs_count, plan.steps, nslots, (int)q->literals.size(), dummy, nullptr, &ct);
    if (ct != total_tiles) return fail(PA_EINVAL, "internal: count pass tiles differ");
    DevQuery& c = q->hq_count;
    c = q->hq;
    c.strategy = q->count_strat;
    c.count_skip_gb = q->count_skip;
    c.image_dwords_max = count_plan.img_dw;
    c.ring = count_plan.ring;
    c.dma_per_tile = count_plan.dma;
    c.num_staged = 0;
    for (int sl = 0; sl < nslots; ++sl) {
      bool st = false;
      for (const DevSeg& d : q->hsegs_count) st |= d.cols[sl].lds_off >= 0;
      if (st) c.staged_slots[c.num_staged++] = sl;
    }
    c.lds_acc_bytes = (uint32_t)(((size_t)q->hq.num_parts * 4 + 15) & ~(size_t)15);
    q->count_lds = (int)count_plan.lds;
    q->count_ring = count_plan.ring;
    // the count pass stages fewer columns, so more of its workgroups fit a CU: k per emit workgroup (each walks 1/k of
    // that workgroup's tiles; part_scan_kernel sums their rows), as many as are resident at once
    q->count_k = std::max(1, count_plan.wg_per_cu / std::max(1, wg_cu));
    while (q->count_k > 1 && (int64_t)q->grid * q->count_k * kWavesPerWG > total_tiles) --q->count_k;
    // the emit pass's LDS: partition bin state + bins in front of the ring
    q->hq.lds_acc_bytes = (uint32_t)(plan.lds - (size_t)wpw * plan.ring * plan.img_dw * 4);
    if (q->split_emit) {  // the H launch: same tiles and staging, its own ring depth, bins and partitions
      DevQuery& e = q->hq_h;
      e = q->hq;
      e.strategy = STRAT_PEMIT;
      e.ring = q->emit_h_ring;
      e.lds_acc_bytes = (uint32_t)((size_t)q->emit_h_lds -
                                   (size_t)scan_waves(q->emit_h_strat) * q->emit_h_ring * plan.img_dw * 4);
      e.part_lo = q->hq.pv;
      e.part_hi = q->hq.num_parts;
    }
    rc = plan_scratch(q, P);
    if (rc) return rc;
  }
  if (q->limit_mode) {
    rc = plan_limit_buffers(q, P, cus, total_tiles);
    if (rc) return rc;
  }
  rc = alloc_leaps(q, P);
  if (rc) return rc;
  rc = upload_descriptors(q);
  if (rc) return rc;
  rc = jit_plan(q, P, cus);
  if (rc) return rc;
  rc = pve_plan(q, P, cus);
  if (rc) return rc;
  PA_HIP(hipDeviceSynchronize());
  q->prepared = true;
  return PA_OK;
}

int64_t pa_query_num_keys(const pa_query* q) { return q ? q->num_keys : -1; }

int pa_query_reset(pa_query* q, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  hipStream_t st = (hipStream_t)stream;
  // one memset of the whole accumulator block, then the MIN/MAX sections to their identities
  PA_HIP(hipMemsetAsync(q->external_acc ? q->external_acc : q->acc.p, 0, q->acc.n, st));
  if (q->hq.leap_mode) PA_HIP(hipMemsetAsync(q->leap_buf.p, 0, leap_header_bytes(q), st));
  for (const Section& sc : q->sections) {
    if (sc.kind == PA_ACC_MIN_I64 || sc.kind == PA_ACC_KEYS_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MAX, st));
    else if (sc.kind == PA_ACC_MAX_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MIN, st));
  }
  return PA_OK;
}

int pa_query_scan(pa_query* q, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  q->scanned_since_fetch = true;
  if (q->num_tiles == 0) return PA_OK;
  hipStream_t st = (hipStream_t)stream;
  if (q->limit_walk) {  // admitted keys of every segment where the limit can bind, before any pass tests them
    if (q->walk_words > kWalkMaxWords) PA_HIP(hipMemsetAsync(q->lim_admit.p, 0, q->lim_admit.n, st));
    PA_HIP(launch_limit_walk((const DevQuery*)q->dq.p, (const DevSeg*)q->dsegs.p, q->nseg, q->walk_words,
                             q->hq.gb_mv >= 0, st));
  }
  if (q->limit_mode) {  // first-seen positions, per-segment selection of the threshold, admitted aggregation
    const DevQuery* dq = (const DevQuery*)q->dq.p;
    const DevSeg* ds = (const DevSeg*)q->dsegs.p;
    const LimitDesc& F = q->limit;
    const int64_t H = F.fmask + 1;
    PA_HIP(launch_fill_i64((int64_t*)F.fkeys, H, INT64_MAX, st));
    PA_HIP(launch_fill_i64((int64_t*)F.fpos, H, -1, st));
    PA_HIP(launch_fill_i64((int64_t*)F.thresh, std::max(1, q->nseg), -1, st));
    PA_HIP(launch_fill_i64((int64_t*)F.hist, std::max(1, q->nseg) * 128, 0, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 0, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 1, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 2, st));
    return PA_OK;
  }
  if (q->pve.fn) {  // the count-free emit: records in per-workgroup chunks, the partitions' chunk lists, pass C
    if (q->part_vk == kVkGeneric) return fail(PA_EINVAL, "internal: chunk lists need a specialised pass C");
    PartScratch ps{};
    char* vb = (char*)q->pve.buf.p;
    ps.base = (uint64_t*)(vb + q->pve.o_base);
    for (pa_query::PveStream* S : {&q->pve, &q->pvh}) {
      if (!S->fn) continue;
      void* pa = S->args.p;
      void* psg = S->segs.p;
      void* params[] = {&pa, &psg};
      PA_HIP(hipModuleLaunchKernel(S->fn, S->grid, 1, 1, S->waves * kWave, 1, 1, S->lds, st, params, nullptr));
      char* b = (char*)S->buf.p;
      // (the H partitions' bases follow the V partitions' in the V buffer's base array: base[pv + 1 ..])
      uint64_t* base = S == &q->pve ? ps.base : ps.base + q->hq.pv + 1;
      PA_HIP(launch_pve_lists((const uint32_t*)(b + S->o_hist), (uint32_t*)(b + S->o_off), base,
                              (const uint32_t*)(b + S->o_table), (const uint32_t*)(b + S->o_used),
                              (uint32_t*)(b + S->o_index), (uint32_t*)(b + S->o_tot), S->grid, S->parts, S->chunks,
                              S->cr, st));
      if (S == &q->pve) {
        ps.recs_v = (uint32_t*)b;
        ps.chunk_index = (const uint32_t*)(b + S->o_index);
        ps.chunk_shift = __builtin_ctz((unsigned)S->cr);
        ps.chunk_bin_shift = S->bin_shift;
      } else {
        ps.recs_h = (uint32_t*)b;
        ps.chunk_index_h = (const uint32_t*)(b + S->o_index);
        ps.chunk_shift_h = __builtin_ctz((unsigned)S->cr);
        ps.chunk_bin_shift_h = S->bin_shift;
      }
    }
    PA_HIP(launch_part_agg(q->part_vk, (const DevQuery*)q->dq.p, ps, q->pvh.fn ? q->hq.num_parts : q->hq.pv,
                           q->hq.pv, q->hq.v_fmt <= V_FMT_ID, q->part_lds_c, st));
    return PA_OK;
  }
  if (q->partitioned) {  // count pass, range offsets, emit pass into the partitions, per-partition aggregation
    ScratchArena* a = arena_for(q->scratch_dev);
    std::lock_guard<std::mutex> g(a->mu);
    int rc = arena_grow(a, q->sc_bytes);
    if (rc) return rc;
    if (a->used && a->last_stream != st) PA_HIP(hipStreamWaitEvent(st, a->last, 0));
    const PartScratch ps = scratch_of(q, a->p);
    const LmSegPlan* plans = (const LmSegPlan*)q->dplans.p;
    PA_HIP(launch_scan(q->count_strat, q->steps, 0, q->grid * q->count_k, q->count_lds, (const DevQuery*)q->dq_count.p,
                       (const DevSeg*)q->dsegs_count.p, plans, ps, st));
    PA_HIP(launch_part_offsets(&q->hq, ps, q->grid, q->count_k, st));
    PA_HIP(launch_scan(q->emit_strat, q->steps, 0, q->grid, q->lds_bytes, (const DevQuery*)q->dq.p,
                       (const DevSeg*)q->dsegs.p, plans, ps, st));
    if (q->split_emit)
      PA_HIP(launch_scan(q->emit_h_strat, q->steps, 0, q->grid, q->emit_h_lds, (const DevQuery*)q->dq_h.p,
                         (const DevSeg*)q->dsegs.p, plans, ps, st));
    PA_HIP(launch_part_agg(q->part_vk, (const DevQuery*)q->dq.p, ps, q->hq.num_parts, q->hq.pv, q->hq.v_fmt <= V_FMT_ID,
                           q->part_lds_c, st));
    PA_HIP(hipEventRecord(a->last, st));
    a->last_stream = st;
    a->used = true;
    return PA_OK;
  }
  if (q->jit_fn) {  // the query-shape specialised dense kernel
    void* pa = q->jit_args.p;
    void* ps = q->jit_segs.p;
    void* params[] = {&pa, &ps};
    PA_HIP(hipModuleLaunchKernel(q->jit_fn, q->jit_grid, 1, 1, q->jit_waves * kWave, 1, 1, q->jit_lds, st, params,
                                 nullptr));
    return PA_OK;
  }
  PartScratch none{};
  PA_HIP(launch_scan(q->strategy, q->steps, q->lane_major, q->grid, q->lds_bytes, (const DevQuery*)q->dq.p,
                     (const DevSeg*)q->dsegs.p, (const LmSegPlan*)q->dplans.p, none, st));
  q->leap_searched = false;  // (the neighbour searches of the listed E docs run when the statistics are asked for)
  return PA_OK;
}

int pa_query_execute(pa_query* q, void* stream) {
  const int rc = pa_query_reset(q, stream);
  return rc ? rc : pa_query_scan(q, stream);
}

uint64_t pa_query_accumulator_bytes(const pa_query* q) { return q ? (uint64_t)q->acc.n : 0; }

int pa_query_set_accumulator_buffer(pa_query* q, void* device_buffer, uint64_t bytes) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!device_buffer || bytes < q->acc.n) return fail(PA_EINVAL, "accumulator buffer too small");
  if (((uintptr_t)device_buffer & 255) != 0) return fail(PA_EINVAL, "accumulator buffer must be 256-byte aligned");
  char* old = (char*)(q->external_acc ? q->external_acc : q->acc.p);
  char* nb = (char*)device_buffer;
  for (Section& s : q->sections) s.ptr = nb + ((char*)s.ptr - old);
  // every scan descriptor of the query (the partitioned count pass has its own) points into the new block
  auto relocate = [&](DevQuery& h) {
    h.count = (unsigned long long*)(nb + ((char*)h.count - old));
    h.matched_docs = (unsigned long long*)(nb + ((char*)h.matched_docs - old));
    if (q->hashed) h.ht_keys = (long long*)(nb + ((char*)h.ht_keys - old));
    for (int a = 0; a < h.num_aggs; ++a) {
      if (q->agg_section[a] < 0) continue;
      void* p = q->sections[q->agg_section[a]].ptr;
      h.aggs[a].acc_i64 = (int64_t*)p;
      h.aggs[a].acc_f64 = (double*)p;
      h.aggs[a].acc_hll = (uint8_t*)p;
    }
  };
  relocate(q->hq);
  if (q->limit_mode) q->limit.reached = q->hq.matched_docs + 2;
  PA_HIP(hipMemcpy(q->dq.p, &q->hq, sizeof(DevQuery), hipMemcpyHostToDevice));
  if (q->jit_fn) {
    JitArgs a;
    PA_HIP(hipMemcpy(&a, q->jit_args.p, sizeof(a), hipMemcpyDeviceToHost));
    jit_fill_pointers(q, a);
    PA_HIP(hipMemcpy(q->jit_args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  }
  for (pa_query::PveStream* S : {&q->pve, &q->pvh}) {
    if (!S->fn) continue;
    PveArgs a;
    PA_HIP(hipMemcpy(&a, S->args.p, sizeof(a), hipMemcpyDeviceToHost));
    pve_fill_pointers(*S, q->hq.matched_docs, a);
    PA_HIP(hipMemcpy(S->args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  }
  if (q->partitioned) {
    relocate(q->hq_count);
    PA_HIP(hipMemcpy(q->dq_count.p, &q->hq_count, sizeof(DevQuery), hipMemcpyHostToDevice));
    if (q->split_emit) {
      relocate(q->hq_h);
      PA_HIP(hipMemcpy(q->dq_h.p, &q->hq_h, sizeof(DevQuery), hipMemcpyHostToDevice));
    }
  }
  if (!q->external_acc) {
    const size_t n = q->acc.n;
    dev_free(q->acc);
    q->acc.n = n;
  }
  q->external_acc = device_buffer;
  return PA_OK;
}

int32_t pa_query_num_sections(const pa_query* q) { return q ? (int32_t)q->sections.size() : -1; }

void* pa_query_section(const pa_query* q, int32_t section, int32_t* kind, int64_t* num_elements) {
  if (!q || section < 0 || section >= (int32_t)q->sections.size()) {
    fail(PA_EINVAL, "bad section");
    return nullptr;
  }
  if (kind) *kind = q->sections[section].kind;
  if (num_elements) *num_elements = q->sections[section].n;
  return q->sections[section].ptr;
}

int pa_query_stats(const pa_query* q, uint64_t* staged_bytes, uint64_t* num_docs, uint64_t* num_tiles) {
  if (!q) return fail(PA_EINVAL, "null query");
  if (staged_bytes) *staged_bytes = q->staged_bytes;
  if (num_docs) *num_docs = q->num_docs;
  if (num_tiles) *num_tiles = q->num_tiles;
  return PA_OK;
}

int pa_query_plan(const pa_query* q, int32_t* strategy, int32_t* steps, int32_t* dma_slots, int32_t* ring,
                  int32_t* wg_per_cu, int32_t* grid, int32_t* lds_bytes) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  // (the query-shape specialised kernel reports the lane-major dense variant it specialises)
  if (strategy)
    *strategy = q->jit_fn ? (q->jit_waves >= 16 ? STRAT_GDENSE_LM16 : STRAT_GDENSE_LM8)
                          : (q->partitioned ? STRAT_PEMIT : q->strategy);
  if (steps) *steps = q->steps;
  if (dma_slots) *dma_slots = q->dma_slots;
  if (ring) *ring = q->plan_ring;
  if (wg_per_cu) *wg_per_cu = q->plan_wg;
  if (grid) *grid = q->grid;
  if (lds_bytes) *lds_bytes = q->lds_bytes;
  return PA_OK;
}

int32_t pa_query_num_eager_literals(const pa_query* q) { return q && q->prepared ? q->num_eager : -1; }

int32_t pa_query_lane_major(const pa_query* q) { return q && q->prepared ? q->lane_major : -1; }
int32_t pa_query_count_free_emit(const pa_query* q) { return q && q->prepared ? (q->pve.fn ? (q->pvh.fn ? 2 : 1) : 0) : -1; }
int32_t pa_query_partition_keys(const pa_query* q) {
  if (!q || !q->prepared) return -1;
  if (!q->partitioned || q->hq.pv == 0) return 0;
  return q->hq.part_kr_v ? q->hq.part_kr_v : (int32_t)1 << q->hq.kshift_v;
}
int32_t pa_query_dense_packed(const pa_query* q) {
  return q && q->prepared ? (q->jit_fn ? 2 : (q->dense_packed ? 1 : 0)) : -1;
}

int32_t pa_query_column_staged(const pa_query* q, int32_t column_id) {
  if (!q || !q->prepared || q->nseg == 0) return -1;
  for (size_t sl = 0; sl < q->slot_cols.size(); ++sl)
    if (q->slot_cols[sl] == column_id) {
      if (q->jit_fn) return std::count(q->jit_cols.begin(), q->jit_cols.end(), (int)sl) ? 1 : 0;
      return q->hsegs[0].cols[sl].lds_off >= 0 ? 1 : 0;
    }
  return -1;
}

int64_t pa_query_matched_docs(const pa_query* q) { return q && q->prepared ? q->last_matched : -1; }

// ---------------------------------------------------------------- cross-GPU merge of hashed key spaces
int32_t pa_query_limit_trimming(const pa_query* q) {
  return q && q->prepared ? (q->limit_mode ? 1 : (q->limit_walk ? 2 : 0)) : -1;
}

int64_t pa_query_num_groups_limit_reached(const pa_query* q) { return q && q->prepared ? q->last_reached : -1; }

int pa_query_key_layout(const pa_query* q, int32_t* hashed, int32_t* shifts) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (hashed) *hashed = q->hashed ? 1 : 0;
  if (shifts)
    for (int j = 0; j < q->spec.num_group_by; ++j) shifts[j] = q->hashed ? q->key_shift[j] : 0;
  return PA_OK;
}

int32_t pa_query_key_words(const pa_query* q) { return q && q->prepared ? (q->hashed ? q->key_words : 1) : -1; }

void pa_query_destroy(pa_query* q) { delete q; }

}  // extern "C"
