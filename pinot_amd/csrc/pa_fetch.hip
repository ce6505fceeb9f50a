// Results: pa_query_fetch (compaction of the non-empty keys, one DMA per column) and the hashed key space's row
// pack / merge for the cross-GPU exchange.
#include "pa_host.h"

extern "C" {
int64_t pa_query_fetch(pa_query* q, void* stream, int64_t capacity, int64_t* out_keys, int64_t* out_counts,
                       void* const* out_aggs) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  hipStream_t st = (hipStream_t)stream;
  const pa_query_spec& s = q->spec;
  const int64_t K = q->num_keys;
  const bool grouped = s.num_group_by != 0;
  char* dbase = (char*)(q->external_acc ? q->external_acc : q->acc.p);

  // Decodes `nrows` host rows into the caller's arrays: row r has key key_of(r, w) (word w < kw: two-word hashed keys
  // fill out_keys[2 n], out_keys[2 n + 1]), count hc[r] and the aggregation section rows at sec(section)[r * per]. Rows
  // with a zero count are skipped when `skip_empty`. `order` (optional) lists the rows to emit, in output order (hashed
  // key spaces: sorted by packed key).
  const int kw = q->hashed ? q->key_words : 1;
  auto decode = [&](int64_t nrows, const uint64_t* hc, const std::function<const char*(int)>& sec,
                    const std::function<int64_t(int64_t, int)>& key_of, bool skip_empty,
                    const std::vector<int64_t>* order) -> int64_t {
    const char* asec[PA_MAX_AGGS];  // section base per aggregation, resolved once (not per row)
    for (int a = 0; a < s.num_aggs; ++a) asec[a] = q->agg_section[a] >= 0 ? sec(q->agg_section[a]) : nullptr;
    int64_t n = 0;
    const int64_t total = order ? (int64_t)order->size() : nrows;
    for (int64_t oi = 0; oi < total; ++oi) {
      const int64_t r = order ? (*order)[oi] : oi;
      if (skip_empty && hc[r] == 0) continue;
      if (n < capacity) {
        if (out_keys)
          for (int w = 0; w < kw; ++w) out_keys[kw * n + w] = key_of(r, w);
        if (out_counts) out_counts[n] = (int64_t)hc[r];
        for (int a = 0; a < s.num_aggs; ++a) {
          if (!out_aggs || !out_aggs[a]) continue;
          const pa_agg_spec& A = s.aggs[a];
          double* outd = (double*)out_aggs[a];
          if (A.type == PA_AGG_COUNT) {
            outd[n] = (double)hc[r];
            continue;
          }
          const char* sp = asec[a];
          const int src = q->hq.aggs[a].src;
          if (A.type == PA_AGG_DISTINCTCOUNTHLL || A.type == PA_AGG_DISTINCTCOUNT) {
            const int64_t per = A.type == PA_AGG_DISTINCTCOUNT ? presence_stride(A) : int64_t(1) << A.log2m;
            uint8_t* o = (uint8_t*)out_aggs[a] + n * per;
            std::memcpy(o, (const uint8_t*)sp + r * per, (size_t)per);
          } else if (A.type == PA_AGG_SUM || A.type == PA_AGG_COUNT_MV) {
            const int64_t* hv = (const int64_t*)sp;
            // SRC_LONG: exact 96-bit total, rounded once (the reference's double of the exact sum)
            if (src == SRC_LONG) outd[n] = (double)(((__int128)hv[2 * r + 1] << 32) + (__int128)(uint64_t)hv[2 * r]);
            else outd[n] = src == SRC_INT ? (double)hv[r] : ((const double*)sp)[r];
          } else {  // MIN / MAX; empty aggregation-only result -> +/-inf (Min/MaxAggregationFunction DEFAULT_VALUE)
            const int64_t e8 = ((const int64_t*)sp)[r];
            if (hc[r] == 0) outd[n] = A.type == PA_AGG_MIN ? __builtin_inf() : -__builtin_inf();
            else outd[n] = src != SRC_DOUBLE ? (double)e8 : f64_order_decode(e8);
          }
        }
      }
      ++n;
    }
    return n;
  };

  // Small accumulator blocks (the common case: a few thousand keys): ONE device-to-host copy of the whole block into
  // pinned memory and one synchronisation, then compaction + decode on the host.
  if (q->acc.n <= kFetchWholeBlockBytes) {
    if (!q->host_acc) {
      if (hipHostMalloc(&q->host_acc, std::max<size_t>(q->acc.n, 16), hipHostMallocDefault) != hipSuccess) {
        q->host_acc = nullptr;
        return fail(PA_ENOMEM, "hipHostMalloc for the accumulator copy failed");
      }
    }
    PA_HIP(hipMemcpyAsync(q->host_acc, dbase, q->acc.n, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    const char* hb = (const char*)q->host_acc;
    auto hsec = [&](int sec) { return hb + ((char*)q->sections[sec].ptr - dbase); };
    const uint64_t* docs = (const uint64_t*)hsec((int)q->sections.size() - 1);
    q->last_matched = (int64_t)docs[0];
    q->last_reached = (int64_t)docs[2];
    q->scanned_since_fetch = false;
    if (docs[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
    if (docs[3]) return fail(PA_EHIP, "internal: partitioned passes disagree on record counts");
    const uint64_t* hc = (const uint64_t*)hsec(0);
    if (q->hashed) {
      const int64_t* hk = (const int64_t*)hsec(q->keys_section);
      const int ks = kw == 2 ? 3 : 1;  // key-section words per slot
      std::vector<int64_t> order;
      for (int64_t r = 0; r < K; ++r)
        if (hc[r]) order.push_back(r);
      std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return hk[ks * a] != hk[ks * b] ? hk[ks * a] < hk[ks * b] : (kw == 2 && hk[ks * a + 1] < hk[ks * b + 1]);
      });
      return decode(K, hc, hsec, [&](int64_t r, int w) { return hk[ks * r + w]; }, false, &order);
    }
    return decode(K, hc, hsec, [](int64_t r, int) { return r; }, grouped, nullptr);
  }

  // Large key spaces: ordered compaction of the non-empty keys on the GPU (count + scan, then key ids and every
  // section's rows gathered into a staging block), one copy of the compacted rows, decode on the host.
  const int64_t nb = (K + 2047) / 2048;
  if ((int64_t)q->fetch_blocks.n < (nb + 1) * 4) {
    dev_free(q->fetch_blocks);
    int rc = dev_alloc(q->fetch_blocks, (size_t)(nb + 1) * 4);
    if (rc) return rc;
  }
  const int all = grouped ? 0 : 1;
  uint32_t total = 0;
  uint64_t md[4] = {0, 0, 0, 0};
  PA_HIP(launch_compact((const unsigned long long*)q->sections[0].ptr, K, all, (uint32_t*)q->fetch_blocks.p, 0,
                        nullptr, 0, st));
  PA_HIP(hipMemcpyAsync(&total, (uint32_t*)q->fetch_blocks.p + nb, 4, hipMemcpyDeviceToHost, st));
  PA_HIP(hipMemcpyAsync(md, q->sections.back().ptr, 32, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  q->last_matched = (int64_t)md[0];
  q->last_reached = (int64_t)md[2];
  q->scanned_since_fetch = false;
  if (md[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
  if (md[3]) return fail(PA_EHIP, "internal: partitioned passes disagree on record counts");
  const int64_t m = (int64_t)total;
  const int64_t rows_cap = std::min<int64_t>(m, std::max<int64_t>(capacity, 0));
  if (rows_cap == 0) return m;
  if (!q->hashed) {
    // Direct key space: the compaction writes the caller's representation (key ids, counts, doubles / register bytes)
    // into staging columns on the GPU, and each column goes to the caller's array in one copy (a DMA straight into
    // pinned memory when the caller's arrays are pinned: engine.py keeps a reused pinned output pool). No host decode.
    FinalDesc f;
    std::memset(&f, 0, sizeof(f));
    f.nagg = s.num_aggs;
    std::vector<size_t> off(s.num_aggs, 0);
    size_t bytes = ((size_t)rows_cap * 16 + 255) & ~(size_t)255;  // keys | counts
    for (int a = 0; a < s.num_aggs; ++a) {
      const pa_agg_spec& A = s.aggs[a];
      f.type[a] = A.type;
      f.src[a] = q->hq.aggs[a].src;
      f.sec[a] = q->agg_section[a] >= 0 ? q->sections[q->agg_section[a]].ptr : nullptr;
      f.per[a] = A.type == PA_AGG_DISTINCTCOUNT ? presence_stride(A)
                                                : (A.type == PA_AGG_DISTINCTCOUNTHLL ? (int64_t(1) << A.log2m) : 8);
      off[a] = bytes;
      bytes += ((size_t)rows_cap * (size_t)f.per[a] + 255) & ~(size_t)255;
    }
    if (q->fetch_stage.n < bytes) {
      dev_free(q->fetch_stage);
      int rc = dev_alloc(q->fetch_stage, bytes);
      if (rc) return rc;
    }
    char* ds = (char*)q->fetch_stage.p;
    f.keys = (int64_t*)ds;
    f.counts = (int64_t*)(ds + (size_t)rows_cap * 8);
    for (int a = 0; a < s.num_aggs; ++a) f.out[a] = ds + off[a];
    PA_HIP(launch_compact_final((const unsigned long long*)q->sections[0].ptr, K, all,
                                (const uint32_t*)q->fetch_blocks.p, rows_cap, &f, st));
    if (out_keys) PA_HIP(hipMemcpyAsync(out_keys, f.keys, (size_t)rows_cap * 8, hipMemcpyDeviceToHost, st));
    if (out_counts) PA_HIP(hipMemcpyAsync(out_counts, f.counts, (size_t)rows_cap * 8, hipMemcpyDeviceToHost, st));
    for (int a = 0; a < s.num_aggs; ++a)
      if (out_aggs && out_aggs[a])
        PA_HIP(hipMemcpyAsync(out_aggs[a], f.out[a], (size_t)rows_cap * (size_t)f.per[a], hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    return m;
  }
  // staging: keys | count | one block per aggregation section (rows x per x es), 256-byte aligned pieces
  CompactDesc d;
  std::memset(&d, 0, sizeof(d));
  std::vector<int> secs = {0};
  for (int a = 0; a < s.num_aggs; ++a)
    if (q->agg_section[a] >= 0) secs.push_back(q->agg_section[a]);
  if (q->hashed) secs.push_back(q->keys_section);
  // hashed key spaces: every non-empty slot is needed to sort by packed key before the capacity cut
  const int64_t rows_needed = q->hashed ? m : std::min<int64_t>(m, std::max<int64_t>(capacity, 0));
  std::vector<size_t> offs;
  const int64_t rows = rows_needed;
  size_t bytes = ((size_t)rows * 8 + 255) & ~(size_t)255;
  for (int sec : secs) {
    const Section& sc = q->sections[sec];
    const int es = (int)section_es(sc.kind);  // HLL registers / presence: one byte each
    const int64_t per = sc.n / K;
    offs.push_back(bytes);
    bytes += ((size_t)rows * per * es + 255) & ~(size_t)255;
  }
  if (q->fetch_stage.n < bytes) {
    dev_free(q->fetch_stage);
    int rc = dev_alloc(q->fetch_stage, bytes);
    if (rc) return rc;
    if (q->fetch_host) (void)hipHostFree(q->fetch_host);
    if (hipHostMalloc(&q->fetch_host, bytes, hipHostMallocDefault) != hipSuccess) {
      q->fetch_host = nullptr;
      return fail(PA_ENOMEM, "hipHostMalloc for the fetch staging failed");
    }
  }
  char* dstage = (char*)q->fetch_stage.p;
  d.nsec = (int32_t)secs.size();
  d.keys = (int64_t*)dstage;
  for (size_t i = 0; i < secs.size(); ++i) {
    const Section& sc = q->sections[secs[i]];
    d.es[i] = (int32_t)section_es(sc.kind);
    d.per[i] = sc.n / K;
    d.src[i] = sc.ptr;
    d.dst[i] = dstage + offs[i];
  }
  PA_HIP(launch_compact((const unsigned long long*)q->sections[0].ptr, K, all, (uint32_t*)q->fetch_blocks.p, rows,
                        &d, 1, st));
  PA_HIP(hipMemcpyAsync(q->fetch_host, dstage, bytes, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  const char* hb = (const char*)q->fetch_host;
  const int64_t* hkeys = (const int64_t*)hb;
  std::map<int, const char*> hsec;
  for (size_t i = 0; i < secs.size(); ++i) hsec[secs[i]] = hb + offs[i];
  if (q->hashed) {  // rows are slots: emit them in packed-key order
    const int64_t* pk = (const int64_t*)hsec[q->keys_section];
    const int ks = kw == 2 ? 3 : 1;
    std::vector<int64_t> order(rows);
    for (int64_t r = 0; r < rows; ++r) order[r] = r;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      return pk[ks * a] != pk[ks * b] ? pk[ks * a] < pk[ks * b] : (kw == 2 && pk[ks * a + 1] < pk[ks * b + 1]);
    });
    order.resize(rows_cap);
    decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; },
           [&](int64_t r, int w) { return pk[ks * r + w]; }, false, &order);
    return m;
  }
  decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; }, [&](int64_t r, int) { return hkeys[r]; },
         false, nullptr);
  return m;
}

// The row layout of a hashed block: every per-key section (numDocsScanned counters excluded) in section order.
static int row_desc(const pa_query* q, RowDesc& d) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!q->hashed || q->keys_section < 0) return fail(PA_EINVAL, "row merge needs a hashed key space");
  std::memset(&d, 0, sizeof(d));
  int64_t off = 0;
  for (const Section& sc : q->sections) {
    if (sc.kind == PA_ACC_DOCS_U64) continue;
    if (d.nsec >= kMaxRowSecs) return fail(PA_EINVAL, "internal: too many sections for a row");
    RowSec& r = d.sec[d.nsec++];
    switch (sc.kind) {
      case PA_ACC_SUM_F64: r.op = ROW_ADD_F64; break;
      case PA_ACC_MIN_I64: r.op = ROW_MIN_I64; break;
      case PA_ACC_MAX_I64: r.op = ROW_MAX_I64; break;
      case PA_ACC_HLL_U8: case PA_ACC_PRESENCE_U8: r.op = ROW_MAX_U8; break;
      case PA_ACC_KEYS_I64: r.op = ROW_KEY; break;
      default: r.op = ROW_ADD_U64; break;  // COUNT, SUM (int64 and the exact lo / hi pair)
    }
    r.slot_bytes = sc.n / q->num_keys * (int64_t)section_es(sc.kind);
    if (r.slot_bytes % 8) return fail(PA_EINVAL, "internal: row section not a multiple of 8 bytes");
    r.row_off = off;
    r.base = sc.ptr;
    if (sc.kind == PA_ACC_KEYS_I64) {
      d.key_off = off;
      d.keys = (long long*)sc.ptr;
    }
    if (sc.kind == PA_ACC_COUNT_U64) d.count = (const unsigned long long*)sc.ptr;
    off += r.slot_bytes;
  }
  d.row_bytes = off;
  d.num_slots = q->num_keys;
  d.ht_mask = q->ht_slots - 1;
  d.key_words = q->key_words;
  return PA_OK;
}

static int merge_scratch(pa_query* q, size_t bytes) {
  if (q->merge_buf.n >= bytes) return PA_OK;
  dev_free(q->merge_buf);
  return dev_alloc(q->merge_buf, bytes);
}

int64_t pa_query_row_bytes(const pa_query* q) {
  RowDesc d;
  const int rc = row_desc(q, d);
  return rc ? rc : d.row_bytes;
}

int pa_query_pack_rows(pa_query* q, int32_t world, void* device_rows, int64_t* counts, void* stream) {
  RowDesc d;
  int rc = row_desc(q, d);
  if (rc) return rc;
  if (world < 1 || world > 1024 || !counts) return fail(PA_EINVAL, "pack rows: bad world size or null counts");
  hipStream_t st = (hipStream_t)stream;
  // scratch: counts[world], cursor[world], row_slot[num_slots]
  rc = merge_scratch(q, (size_t)(2 * world + d.num_slots) * 8);
  if (rc) return rc;
  unsigned long long* cnt = (unsigned long long*)q->merge_buf.p;
  unsigned long long* cur = cnt + world;
  int64_t* row_slot = (int64_t*)(cur + world);
  PA_HIP(hipMemsetAsync(cnt, 0, (size_t)world * 8, st));
  PA_HIP(launch_pack_index(d, world, 0, cnt, nullptr, nullptr, st));
  std::vector<unsigned long long> h(world);
  PA_HIP(hipMemcpyAsync(h.data(), cnt, (size_t)world * 8, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  int64_t total = 0;
  std::vector<unsigned long long> start(world);
  for (int r = 0; r < world; ++r) {
    counts[r] = (int64_t)h[r];
    start[r] = (unsigned long long)total;
    total += (int64_t)h[r];
  }
  if (!device_rows || total == 0) return PA_OK;
  PA_HIP(hipMemcpyAsync(cur, start.data(), (size_t)world * 8, hipMemcpyHostToDevice, st));
  PA_HIP(launch_pack_index(d, world, 1, nullptr, cur, row_slot, st));
  PA_HIP(launch_pack_copy(d, row_slot, total, (unsigned char*)device_rows, st));
  PA_HIP(hipStreamSynchronize(st));
  return PA_OK;
}

int pa_query_merge_rows(pa_query* q, const void* device_rows, int64_t num_rows, int64_t* groups, int64_t* overflow,
                        void* stream) {
  RowDesc d;
  int rc = row_desc(q, d);
  if (rc) return rc;
  if (num_rows < 0 || (num_rows > 0 && !device_rows)) return fail(PA_EINVAL, "merge rows: bad rows");
  hipStream_t st = (hipStream_t)stream;
  rc = merge_scratch(q, (size_t)(8 + std::max<int64_t>(num_rows, d.num_slots)) * 8);
  if (rc) return rc;
  unsigned long long* ctr = (unsigned long long*)q->merge_buf.p;
  int64_t* row_slot = (int64_t*)(ctr + 8);
  // the block is reset except its numDocsScanned counters, which stay this rank's (the broker sums them)
  void* docs = q->sections.back().ptr;
  PA_HIP(hipMemcpyAsync(ctr + 4, docs, 32, hipMemcpyDeviceToDevice, st));
  rc = pa_query_reset(q, stream);
  if (rc) return rc;
  PA_HIP(hipMemcpyAsync(docs, ctr + 4, 32, hipMemcpyDeviceToDevice, st));
  PA_HIP(hipMemsetAsync(ctr, 0, 32, st));
  PA_HIP(launch_merge_rows(d, (const unsigned char*)device_rows, num_rows, row_slot, ctr, st));
  unsigned long long h[4];
  PA_HIP(hipMemcpyAsync(h, ctr, 32, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  if (groups) *groups = (int64_t)h[0];
  if (overflow) *overflow = (int64_t)h[1];
  return PA_OK;
}

}  // extern "C"
