// Filter statistics on the host side: GPU leaf bitmaps and filter counts, the fused leap counts, and the
// execution-statistics engine (pa_query_execution_stats) over the reference's operator trees.
#include "pa_host.h"

extern "C" {
// words per leaf bitmap: whole 64-doc steps, rounded up to 4 words (the count kernels read 16-byte groups)
int64_t leaf_words(int64_t num_docs) { return (num_docs + 127) / 128 * 4; }

int64_t pa_query_leaf_bitmap_words(const pa_query* q, int32_t segment) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (segment < 0 || segment >= q->nseg) return fail(PA_EINVAL, "segment index out of range");
  return leaf_words((int64_t)q->segs[segment]->num_docs);
}

int pa_query_leaf_bitmaps(pa_query* q, int32_t segment, uint32_t* device_out, void* stream) {
  const int64_t words = pa_query_leaf_bitmap_words(q, segment);
  if (words < 0) return (int)words;
  if (!device_out) return fail(PA_EINVAL, "null bitmap buffer");
  hipStream_t st = (hipStream_t)stream;
  const DevSeg* ds = (const DevSeg*)q->dsegs.p + segment;
  for (int l = 0; l < q->spec.num_leaves; ++l) {
    // the leaf's first CNF literal: literal value = leaf value XOR the literal's negation
    int li = -1;
    for (size_t i = 0; i < q->literals.size() && li < 0; ++i)
      if (q->literals[i].leaf == l) li = (int)i;
    if (li < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
    PA_HIP(launch_leaf_bitmap(ds, li, q->literals[li].neg ? 1 : 0, q->segs[segment]->num_docs,
                              device_out + (size_t)l * words, st));
  }
  return PA_OK;
}

// Validated postfix program of pa_bitmap_counts / pa_query_filter_counts into tok[0..len).
int check_bit_prog(const int32_t* prog, int32_t len, int32_t num_leaves, bool required, int32_t* tok) {
  if (len < 0 || len > kBitProgMax || (required && len == 0) || (len > 0 && !prog))
    return fail(PA_EINVAL, "bitmap program length out of range");
  int depth = 0;
  for (int i = 0; i < len; ++i) {
    const int32_t t = prog[i];
    if (t >= 0) {
      if (t >= num_leaves) return fail(PA_EINVAL, "bitmap program names a leaf out of range");
      if (++depth > kBitProgStack) return fail(PA_EINVAL, "bitmap program too deep");
    } else if (t == PA_BIT_NOT) {
      if (depth < 1) return fail(PA_EINVAL, "bitmap program: NOT on an empty stack");
    } else if (t == PA_BIT_AND || t == PA_BIT_OR) {
      if (depth < 2) return fail(PA_EINVAL, "bitmap program: AND/OR needs two masks");
      --depth;
    } else {
      return fail(PA_EINVAL, "bitmap program: unknown token");
    }
    tok[i] = t;
  }
  if (len > 0 && depth != 1) return fail(PA_EINVAL, "bitmap program must leave exactly one mask");
  return PA_OK;
}

constexpr size_t kBitTokBytes = 2 * kBitProgMax * 4;

// The count kernels keep up to 4 leaves' words in registers: renumber the programs' leaf tokens to positions in
// job.uleaf when they use at most 4 distinct leaves (else nu = 0: leaf ids, loaded in program order).
void renumber_leaves(BitJob& job, int32_t* tok) {
  int32_t u[4];
  int nu = 0;
  const int lens[2] = {job.len_a, job.len_b};
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < lens[k]; ++i) {
      const int32_t t = tok[k * kBitProgMax + i];
      if (t < 0) continue;
      int p = 0;
      while (p < nu && u[p] != t) ++p;
      if (p == nu) {
        if (nu == 4) {
          job.nu = 0;
          return;
        }
        u[nu++] = t;
      }
    }
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < lens[k]; ++i) {
      int32_t& t = tok[k * kBitProgMax + i];
      if (t < 0) continue;
      int p = 0;
      while (u[p] != t) ++p;
      t = p;
    }
  job.nu = nu;
  for (int p = 0; p < 4; ++p) job.uleaf[p] = p < nu ? u[p] : 0;
}

BitJob make_bit_job(const uint32_t* bm, int64_t words, int64_t num_docs, int64_t first_block, const int32_t* tok,
                    int32_t len_a, int32_t len_b, uint32_t* scratch, int64_t* out) {
  BitJob j{};
  j.bm = bm;
  j.words = words;
  j.num_docs = num_docs;
  j.first_block = first_block;
  j.nb = bit_count_blocks(num_docs);
  j.tok = tok;
  j.len_a = len_a;
  j.len_b = len_b;
  j.scratch = scratch;
  // the partial counts after block_last / block_in, 8-byte aligned (bit_count_scratch_words: 10 words per workgroup)
  j.part = scratch ? (unsigned long long*)(((uintptr_t)(scratch + 2 * j.nb) + 7) & ~(uintptr_t)7) : nullptr;
  j.out = (unsigned long long*)out;
  return j;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int64_t pa_bitmap_counts_scratch_bytes(int64_t words) {
  if (words < 0) return fail(PA_EINVAL, "negative word count");
  return (int64_t)(align256(4 * (size_t)bit_count_scratch_words(words)) + align256(4 * (size_t)bit_count_blocks(32 * words)) +
                   align256(sizeof(BitJob)) + kBitTokBytes);
}

int pa_bitmap_counts(const uint32_t* device_bitmaps, int64_t words, int32_t num_leaves, int64_t num_docs,
                     const int32_t* prog_a, int32_t len_a, const int32_t* prog_b, int32_t len_b, void* device_scratch,
                     int64_t* device_out, void* stream) {
  if (!device_out || num_docs < 0 || words < (num_docs + 31) / 32 || words % 4 != 0)
    return fail(PA_EINVAL, "bad bitmap counts arguments (words: a multiple of 4 covering num_docs)");
  if (num_docs > 0 && !device_bitmaps) return fail(PA_EINVAL, "null bitmaps");
  struct {
    BitJob job;
    int32_t tok[2 * kBitProgMax];
  } h{};
  int rc = check_bit_prog(prog_a, len_a, num_leaves, true, h.tok);
  if (!rc) rc = check_bit_prog(prog_b, len_b, num_leaves, false, h.tok + kBitProgMax);
  if (rc) return rc;
  if (num_docs == 0) return PA_OK;
  if (!device_scratch) return fail(PA_EINVAL, "null scratch");
  char* sc = (char*)device_scratch;
  const size_t off_table = align256(4 * (size_t)bit_count_scratch_words(words));
  const size_t off_job = off_table + align256(4 * (size_t)bit_count_blocks(32 * words));
  const size_t off_tok = off_job + align256(sizeof(BitJob));
  h.job = make_bit_job(device_bitmaps, words, num_docs, 0, (const int32_t*)(sc + off_tok), len_a, len_b,
                       (uint32_t*)sc, device_out);
  renumber_leaves(h.job, h.tok);
  hipStream_t st = (hipStream_t)stream;
  PA_HIP(hipMemcpyAsync(sc + off_job, &h.job, sizeof(BitJob), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemcpyAsync(sc + off_tok, h.tok, kBitTokBytes, hipMemcpyHostToDevice, st));
  PA_HIP(launch_bit_counts_batch((const BitJob*)(sc + off_job), 1, h.job.nb, len_b > 0, (int32_t*)(sc + off_table), st));
  PA_HIP(hipStreamSynchronize(st));  // (the host staging above is on this stack frame)
  return PA_OK;
}

int pa_query_filter_counts(pa_query* q, int32_t num_requests, const int32_t* segments, const int32_t* programs,
                           const int32_t* lengths, int64_t* out, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (num_requests < 0 || (num_requests > 0 && (!segments || !programs || !lengths || !out)))
    return fail(PA_EINVAL, "bad filter counts arguments");
  if (num_requests == 0) return PA_OK;
  const int nl = q->spec.num_leaves;
  std::vector<int> leaf_lit(nl, -1);
  for (int l = 0; l < nl; ++l) {
    for (size_t i = 0; i < q->literals.size() && leaf_lit[l] < 0; ++i)
      if (q->literals[i].leaf == l) leaf_lit[l] = (int)i;
    if (leaf_lit[l] < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
  }
  // device layout: leaf bitmaps of every requested segment | per-request scratch | counts | jobs | leaf jobs | tokens
  std::vector<int64_t> bm_off(q->nseg, -1);
  size_t bm_words = 0;
  for (int r = 0; r < num_requests; ++r) {
    const int si = segments[r];
    if (si < 0 || si >= q->nseg) return fail(PA_EINVAL, "request names a segment out of range");
    if (bm_off[si] < 0) {
      bm_off[si] = (int64_t)bm_words;
      bm_words += (size_t)nl * (size_t)leaf_words(q->segs[si]->num_docs);
    }
  }
  std::vector<int64_t> sc_off(num_requests);
  size_t sc_words = 0;
  std::vector<BitJob> jobs(num_requests);
  std::vector<int32_t> tok((size_t)num_requests * 2 * kBitProgMax, 0);
  bool any_b = false;
  int64_t blocks = 0;
  for (int r = 0; r < num_requests; ++r) {
    int32_t* t = tok.data() + (size_t)r * 2 * kBitProgMax;
    const int la = lengths[2 * r], lb = lengths[2 * r + 1];
    int rc = check_bit_prog(programs + (size_t)r * 2 * kBitProgMax, la, nl, true, t);
    if (!rc) rc = check_bit_prog(programs + (size_t)r * 2 * kBitProgMax + kBitProgMax, lb, nl, false, t + kBitProgMax);
    if (rc) return rc;
    any_b |= lb > 0;
    const int64_t n = q->segs[segments[r]]->num_docs;
    const int64_t words = leaf_words(n);
    sc_off[r] = (int64_t)sc_words;
    sc_words += (size_t)bit_count_scratch_words(words);
    jobs[r] = make_bit_job(nullptr, words, n, blocks, nullptr, la, lb, nullptr, nullptr);
    renumber_leaves(jobs[r], t);
    blocks += jobs[r].nb;
  }
  std::vector<LeafJob> ljobs;
  int64_t lblocks = 0;
  for (int si = 0; si < q->nseg; ++si) {
    if (bm_off[si] < 0 || q->segs[si]->num_docs == 0) continue;
    const int64_t n = q->segs[si]->num_docs, words = leaf_words(n);
    for (int l = 0; l < nl; ++l) {
      ljobs.push_back(LeafJob{(const DevSeg*)q->dsegs.p + si, nullptr, n, lblocks, leaf_lit[l],
                              q->literals[leaf_lit[l]].neg ? 1 : 0});
      ljobs.back().out = (uint32_t*)(intptr_t)(bm_off[si] + (int64_t)l * words);  // (word offset; rebased below)
      lblocks += leaf_bitmap_blocks(n);
    }
  }
  const size_t o_bm = 0, o_sc = align256(4 * bm_words), o_out = o_sc + align256(4 * sc_words),
               o_jobs = o_out + align256(32 * (size_t)num_requests),
               o_ljobs = o_jobs + align256(sizeof(BitJob) * num_requests),
               o_tok = o_ljobs + align256(sizeof(LeafJob) * std::max<size_t>(1, ljobs.size())),
               o_table = o_tok + align256(4 * tok.size()), total = o_table + 4 * (size_t)std::max<int64_t>(1, blocks);
  if (q->stat_buf.n < total) {
    dev_free(q->stat_buf);
    int rc = dev_alloc(q->stat_buf, total);
    if (rc) return rc;
  }
  char* base = (char*)q->stat_buf.p;
  for (int r = 0; r < num_requests; ++r) {
    jobs[r].bm = (const uint32_t*)(base + o_bm) + bm_off[segments[r]];
    jobs[r].tok = (const int32_t*)(base + o_tok) + (size_t)r * 2 * kBitProgMax;
    jobs[r].scratch = (uint32_t*)(base + o_sc) + sc_off[r];
    jobs[r].part = (unsigned long long*)(((uintptr_t)(jobs[r].scratch + 2 * jobs[r].nb) + 7) & ~(uintptr_t)7);
    jobs[r].out = (unsigned long long*)(base + o_out) + 4 * (size_t)r;
  }
  for (LeafJob& lj : ljobs) lj.out = (uint32_t*)(base + o_bm) + (intptr_t)lj.out;
  hipStream_t st = (hipStream_t)stream;
  PA_HIP(hipMemcpyAsync(base + o_jobs, jobs.data(), sizeof(BitJob) * num_requests, hipMemcpyHostToDevice, st));
  if (!ljobs.empty())
    PA_HIP(hipMemcpyAsync(base + o_ljobs, ljobs.data(), sizeof(LeafJob) * ljobs.size(), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemcpyAsync(base + o_tok, tok.data(), 4 * tok.size(), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemsetAsync(base + o_out, 0, 32 * (size_t)num_requests, st));
  PA_HIP(launch_leaf_bitmaps_batch((const LeafJob*)(base + o_ljobs), (int)ljobs.size(), lblocks, st));
  PA_HIP(launch_bit_counts_batch((const BitJob*)(base + o_jobs), num_requests, blocks, any_b,
                                 (int32_t*)(base + o_table), st));
  PA_HIP(hipMemcpyAsync(out, base + o_out, 32 * (size_t)num_requests, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  return PA_OK;
}

int32_t pa_query_leap_leaf(const pa_query* q) { return q && q->prepared ? q->leap_leaf : -1; }

// the neighbour searches of the E docs the last scan listed (once per scan)
static int leap_search_pending(pa_query* q, hipStream_t st) {
  if (q->hq.leap_mode && !q->leap_searched) {
    PA_HIP(launch_leap_search((const DevQuery*)q->dq.p, (const DevSeg*)q->dsegs.p, q->leap_slices, st));
    q->leap_searched = true;
  }
  return PA_OK;
}

int pa_query_leap_counts(pa_query* q, int64_t* out, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (q->leap_leaf < 0) return fail(PA_EINVAL, "the scan does not count the filter statistics (pa_query_leap_leaf)");
  if (!out) return fail(PA_EINVAL, "null output");
  hipStream_t st = (hipStream_t)stream;
  int rc = leap_search_pending(q, st);
  if (rc) return rc;
  std::vector<int64_t> h((size_t)q->nseg * 3 + 1);
  PA_HIP(hipMemcpyAsync(h.data(), q->leap_buf.p, h.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  const bool overflow = h[(size_t)q->nseg * 3] != 0;  // (a wave's E-doc slice was full: no segment's leaps are known)
  for (int si = 0; si < q->nseg; ++si) {
    out[3 * si] = h[3 * si];
    out[3 * si + 1] = h[3 * si + 1];
    out[3 * si + 2] = (h[3 * si + 2] || overflow) ? 1 : 0;
  }
  return PA_OK;
}

// ---------------------------------------------------------------- execution statistics (pa_query_execution_stats)
// The host's per-segment filter operator trees, reduced as the reference's iterators read them when the projection
// drives the tree's iterator to the end (BlockDocIdSet.iterator() construction + next() until EOF):
//   * a scan driven by next() reads every entry: num_docs, or a multi-value column's values;
//   * OR: OrDocIdIterator drives every child with next() to its end: the children's costs add;
//   * NOT: NotDocIdIterator drives its child with next() to the end and once more: for a leap-frogging AND that call
//     re-runs the chain after its last match (pa_stats.hip "tail");
//   * AND (AndDocIdSet.java:72-186): with index children (sorted / bitmap doc sets) and scan children, or several index
//     children, the index doc sets intersect and each scan's applyAnd reads the docs surviving so far (a popcount of the
//     chain, a value count for a multi-value column); what is left (OR / NOT children) leap-frogs with that doc set
//     first; otherwise every child leap-frogs (AndDocIdIterator), counted on the GPU (pa_stats.hip).
}  // extern "C"

namespace stats {
struct Elem {  // one child iterator of a leap-frog
  int32_t kind = LF_DOCS;
  std::vector<int32_t> prog;
  int32_t mv = -1;
  std::vector<Elem> subs;  // LF_OR: its children (LF_DOCS / LF_SCAN)
};
struct Leap {
  std::vector<Elem> el;
  bool tail = false;
};
struct Plan {
  int64_t cnst = 0;
  std::vector<std::pair<std::vector<int32_t>, int32_t>> counts;  // (doc set, multi-value column or -1)
  std::vector<Leap> leaps;
};
struct Unsupported {};
struct Ctx {
  const pa_query* q;
  int si;
  const pa_filter_op* ops;
  int nops;
  Plan* P;
};

std::vector<int32_t> prog_of(const pa_filter_op& o) { return std::vector<int32_t>(o.prog, o.prog + o.prog_len); }
std::vector<int32_t> prog_join(const std::vector<int32_t>& a, const std::vector<int32_t>& b, int32_t op) {
  if (a.empty()) return b;
  std::vector<int32_t> r(a);
  r.insert(r.end(), b.begin(), b.end());
  r.push_back(op);
  return r;
}

// index after the subtree at i (pre-order), or -1 when malformed
int extent(const pa_filter_op* ops, int nops, int i, int depth = 0) {
  if (i < 0 || i >= nops || depth > 64) return -1;
  int j = i + 1;
  for (int c = 0; c < ops[i].num_children; ++c) {
    j = extent(ops, nops, j, depth + 1);
    if (j < 0) return -1;
  }
  return j;
}
std::vector<int> children(const Ctx& x, int i) {
  std::vector<int> r;
  int j = i + 1;
  for (int c = 0; c < x.ops[i].num_children; ++c) {
    r.push_back(j);
    j = extent(x.ops, x.nops, j);
  }
  return r;
}

const Column* mv_col(const Ctx& x, int32_t col) {
  auto it = x.q->segs[x.si]->cols.find(col);
  if (it == x.q->segs[x.si]->cols.end() || it->second->kind != COL_MV_DICT) throw Unsupported{};
  return it->second;
}

int64_t cost_next(const Ctx& x, int i, bool tail);

// an OR's iterator (OrDocIdSet.java:63-127): more than one sorted child merge into one doc set; nullptr-like result
// (kind LF_DOCS) when that is all of it
bool and_docs_form(const Ctx& x, int i, std::vector<int32_t>* docs);
Elem or_elem(const Ctx& x, int i) {
  Elem e;
  e.kind = LF_OR;
  std::vector<int> kids = children(x, i);
  int nsorted = 0;
  for (int k : kids) nsorted += x.ops[k].kind == PA_FOP_SORTED;
  std::vector<int32_t> merged;
  for (int k : kids) {
    const pa_filter_op& o = x.ops[k];
    if (o.kind == PA_FOP_SORTED && nsorted > 1) {
      merged = prog_join(merged, prog_of(o), PA_BIT_OR);
      continue;
    }
    Elem s;
    std::vector<int32_t> d;
    if (o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP) {
      s.kind = LF_DOCS;
      s.prog = prog_of(o);
    } else if (o.kind == PA_FOP_SCAN) {
      s.kind = LF_SCAN;
      s.prog = prog_of(o);
      if (o.mv_column >= 0) {
        mv_col(x, o.mv_column);
        s.mv = o.mv_column;
      }
    } else if (o.kind == PA_FOP_AND && and_docs_form(x, k, &d)) {
      s.kind = LF_DOCS;  // (its applyAnd reads are counted at construction)
      s.prog = d;
    } else {
      throw Unsupported{};  // an AND / NOT iterator advanced inside an OR inside a leap-frog
    }
    e.subs.push_back(s);
  }
  if (!merged.empty()) {
    Elem s;
    s.kind = LF_DOCS;
    s.prog = merged;
    e.subs.insert(e.subs.begin(), s);
  }
  for (const Elem& s : e.subs) e.prog = prog_join(e.prog, s.prog, PA_BIT_OR);
  if (kids.size() == (size_t)nsorted) {  // every child sorted: one merged doc set
    e.kind = LF_DOCS;
    e.subs.clear();
  }
  return e;
}

// the AND's iterator construction (AndDocIdSet.iterator): applyAnd counts into the plan; returns the leap-frog list
// (empty when the iterator is the merged doc set) and the AND's doc set in *docs
std::vector<Elem> and_build(const Ctx& x, int i, std::vector<int32_t>* docs) {
  std::vector<int> kids = children(x, i);
  std::vector<int> sorted, bitmaps, scans, rest;
  for (int k : kids) {
    const int kd = x.ops[k].kind;
    if (kd == PA_FOP_SORTED) sorted.push_back(k);
    else if (kd == PA_FOP_BITMAP) bitmaps.push_back(k);
    else if (kd == PA_FOP_SCAN) scans.push_back(k);
    else if (kd == PA_FOP_OR) {
      // an OR of sorted children only is one merged (bitmap) doc set
      bool all_sorted = true;
      for (int c : children(x, k)) all_sorted &= x.ops[c].kind == PA_FOP_SORTED;
      if (all_sorted) bitmaps.push_back(k);
      else rest.push_back(k);
    } else {
      rest.push_back(k);
    }
  }
  auto doc_prog = [&](int k) {
    if (x.ops[k].kind != PA_FOP_OR) return prog_of(x.ops[k]);
    std::vector<int32_t> p;
    for (int c : children(x, k)) p = prog_join(p, prog_of(x.ops[c]), PA_BIT_OR);
    return p;
  };
  std::vector<Elem> out;
  docs->clear();
  const size_t nindex = sorted.size() + bitmaps.size();
  if ((nindex > 0 && !scans.empty()) || nindex > 1) {
    std::vector<int32_t> D;
    for (int k : sorted) D = prog_join(D, doc_prog(k), PA_BIT_AND);
    for (int k : bitmaps) D = prog_join(D, doc_prog(k), PA_BIT_AND);
    for (int k : scans) {
      const pa_filter_op& o = x.ops[k];
      if (o.mv_column >= 0) mv_col(x, o.mv_column);
      x.P->counts.push_back({D, o.mv_column});
      D = prog_join(D, prog_of(o), PA_BIT_AND);
    }
    if (rest.empty()) {
      *docs = D;
      return out;
    }
    Elem m;
    m.kind = LF_DOCS;
    m.prog = D;
    out.push_back(m);
    kids = rest;
  }
  for (int k : kids) {
    const pa_filter_op& o = x.ops[k];
    Elem e;
    if (o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP) {
      e.kind = LF_DOCS;
      e.prog = prog_of(o);
    } else if (o.kind == PA_FOP_SCAN) {
      e.kind = LF_SCAN;
      e.prog = prog_of(o);
      if (o.mv_column >= 0) {
        mv_col(x, o.mv_column);
        e.mv = o.mv_column;
      }
    } else if (o.kind == PA_FOP_OR) {
      e = or_elem(x, k);  // (an AND child's iterator is built there: its applyAnd reads)
    } else {
      throw Unsupported{};  // a NOT iterator leap-frogged (next() and advance() mixed on its child)
    }
    out.push_back(e);
  }
  for (const Elem& e : out) *docs = prog_join(*docs, e.prog, PA_BIT_AND);
  return out;
}

bool and_docs_form(const Ctx& x, int i, std::vector<int32_t>* docs) {
  Plan saved = *x.P;
  std::vector<Elem> el = and_build(x, i, docs);
  if (!el.empty()) {
    *x.P = saved;
    return false;
  }
  return true;
}

int64_t cost_next(const Ctx& x, int i, bool tail) {
  const pa_filter_op& o = x.ops[i];
  switch (o.kind) {
    case PA_FOP_EMPTY: case PA_FOP_MATCH_ALL: case PA_FOP_SORTED: case PA_FOP_BITMAP:
      return 0;
    case PA_FOP_SCAN:
      return o.mv_column >= 0 ? mv_col(x, o.mv_column)->total_values : (int64_t)x.q->segs[x.si]->num_docs;
    case PA_FOP_OR: {
      int64_t c = 0;
      for (int k : children(x, i)) c += cost_next(x, k, false);
      return c;
    }
    case PA_FOP_NOT:
      return cost_next(x, i + 1, true);
    case PA_FOP_AND: {
      std::vector<int32_t> d;
      std::vector<Elem> el = and_build(x, i, &d);
      if (el.empty()) return 0;
      size_t nsub = 0;
      for (const Elem& e : el) nsub += e.subs.size();
      if (el.size() > (size_t)kLfMaxK || nsub > (size_t)kLfMaxSub) throw Unsupported{};
      // NotDocIdIterator's extra next(): with an OR child the re-run starts from the OR children's cached answers (a
      // different chain from the first run's last one): not counted here
      if (tail && nsub > 0) throw Unsupported{};
      x.P->leaps.push_back(Leap{el, tail});
      return 0;
    }
  }
  throw Unsupported{};
}

// ---------------------------------------------------------------- iterator replay (stat_replay_kernel)
// The filter shapes the reduction above leaves out are replayed on the GPU, iterator by iterator. The host builds the
// iterator tree BlockDocIdSet.iterator() builds (filter_stats._iterator restated): AndDocIdSet's merge of index children
// and applyAnd over its scan children (counted here, as popcounts), OrDocIdSet's merge of sorted children.
struct RNode {
  int32_t kind = RP_EMPTY;
  bool sorted = false;        // RP_DOCS of a sorted index (the only kind OrDocIdSet merges)
  std::vector<int32_t> prog;  // RP_DOCS / RP_SCAN: the doc set
  int32_t mv = -1;            // RP_SCAN over a multi-value column
  std::vector<int> kids;
};
struct Replay {
  std::vector<RNode> nodes;
  int root = -1;
};

int replay_build(const Ctx& x, int i, Replay& R) {
  const pa_filter_op& o = x.ops[i];
  auto add = [&](RNode n) {
    if (R.nodes.size() >= 4 * (size_t)kRpMaxNodes) throw Unsupported{};
    R.nodes.push_back(std::move(n));
    return (int)R.nodes.size() - 1;
  };
  RNode n;
  switch (o.kind) {
    case PA_FOP_EMPTY:
      n.kind = RP_EMPTY;
      return add(n);
    case PA_FOP_MATCH_ALL:
      n.kind = RP_ALL;
      return add(n);
    case PA_FOP_SORTED:
    case PA_FOP_BITMAP:
      n.kind = RP_DOCS;
      n.sorted = o.kind == PA_FOP_SORTED;
      n.prog = prog_of(o);
      return add(n);
    case PA_FOP_SCAN:
      n.kind = RP_SCAN;
      n.prog = prog_of(o);
      if (o.mv_column >= 0) {
        mv_col(x, o.mv_column);
        n.mv = o.mv_column;
      }
      return add(n);
    case PA_FOP_NOT: {
      const int c = replay_build(x, i + 1, R);
      n.kind = RP_NOT;
      n.kids = {c};
      return add(n);
    }
    default:
      break;
  }
  std::vector<int> its;
  for (int k : children(x, i)) its.push_back(replay_build(x, k, R));
  auto docs = [&](int k) { return R.nodes[k].kind == RP_DOCS; };
  if (o.kind == PA_FOP_OR) {
    // OrDocIdSet.java:63-127: more than one index child merge into one doc set; the reference collects only the sorted
    // ones (its bitmap-based list stays empty), and a bitmap-based child is then neither merged nor kept
    std::vector<int> srt, rest;
    for (int k : its) {
      if (docs(k) && R.nodes[k].sorted) srt.push_back(k);
      if (!docs(k)) rest.push_back(k);
    }
    if (srt.size() > 1) {
      RNode m;
      m.kind = RP_DOCS;
      for (int k : srt) m.prog = prog_join(m.prog, R.nodes[k].prog, PA_BIT_OR);
      const int mi = add(m);
      if (rest.empty()) return mi;
      n.kids = {mi};
      n.kids.insert(n.kids.end(), rest.begin(), rest.end());
    } else {
      n.kids = its;
    }
    n.kind = RP_OR;
    return add(n);
  }
  // AndDocIdSet.java:72-186: index children intersect, each scan child applyAnd-reads the survivors in order
  std::vector<int> idx, scans, rest;
  for (int k : its) {
    if (docs(k)) idx.push_back(k);
    else if (R.nodes[k].kind == RP_SCAN) scans.push_back(k);
    else rest.push_back(k);
  }
  if ((!idx.empty() && !scans.empty()) || idx.size() > 1) {
    std::vector<int32_t> D;
    for (int k : idx) D = prog_join(D, R.nodes[k].prog, PA_BIT_AND);
    for (int k : scans) {
      x.P->counts.push_back({D, R.nodes[k].mv});
      D = prog_join(D, R.nodes[k].prog, PA_BIT_AND);
    }
    RNode m;
    m.kind = RP_DOCS;
    m.prog = D;
    const int mi = add(m);
    if (rest.empty()) return mi;
    n.kids = {mi};
    n.kids.insert(n.kids.end(), rest.begin(), rest.end());
  } else {
    n.kids = its;
  }
  n.kind = RP_AND;
  return add(n);
}

// the reachable tree in pre-order (a node before its children), as the kernel reads it; the programs per node
struct ReplayFlat {
  std::vector<RNode> nodes;  // kids renumbered
  std::vector<int32_t> depth;
};
ReplayFlat replay_flatten(const Replay& R) {
  ReplayFlat F;
  std::function<int(int, int)> emit = [&](int r, int d) -> int {
    if (d >= kRpMaxDepth || F.nodes.size() >= (size_t)kRpMaxNodes) throw Unsupported{};
    const int me = (int)F.nodes.size();
    F.nodes.push_back(R.nodes[r]);
    F.depth.push_back(d);
    std::vector<int> ch;
    for (int c : R.nodes[r].kids) ch.push_back(emit(c, d + 1));
    F.nodes[me].kids = ch;
    return me;
  };
  emit(R.root, 0);
  return F;
}

int check_tree(const pa_filter_op* ops, int nops, int root, int num_leaves) {
  const int end = extent(ops, nops, root);
  if (end < 0) return fail(PA_EINVAL, "execution stats: malformed operator tree");
  for (int i = root; i < end; ++i) {
    const pa_filter_op& o = ops[i];
    const bool leaf = o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP || o.kind == PA_FOP_SCAN;
    if (o.kind < PA_FOP_EMPTY || o.kind > PA_FOP_NOT) return fail(PA_EINVAL, "execution stats: unknown operator kind");
    if ((o.kind == PA_FOP_AND || o.kind == PA_FOP_OR) && o.num_children < 2)
      return fail(PA_EINVAL, "execution stats: AND / OR needs two children");
    if (o.kind == PA_FOP_NOT && o.num_children != 1) return fail(PA_EINVAL, "execution stats: NOT needs one child");
    if ((leaf || o.kind == PA_FOP_EMPTY || o.kind == PA_FOP_MATCH_ALL) && o.num_children != 0)
      return fail(PA_EINVAL, "execution stats: a leaf operator has children");
    if (leaf) {
      int32_t tok[kBitProgMax];
      int rc = check_bit_prog(o.prog, o.prog_len, num_leaves, true, tok);
      if (rc) return rc;
    }
  }
  return PA_OK;
}
}  // namespace stats

extern "C" {

int pa_query_execution_stats(pa_query* q, int32_t num_ops, const pa_filter_op* ops, int32_t num_trees,
                             const int32_t* tree_root, const int32_t* segment_tree, int32_t projected_columns,
                             int64_t docs_scanned, int64_t* out, int64_t* segment_in_filter, void* stream) {
  using namespace stats;
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!out || num_ops < 0 || num_trees < 0 || projected_columns < 0 || (num_ops > 0 && !ops) ||
      (num_trees > 0 && !tree_root) || (q->nseg > 0 && !segment_tree))
    return fail(PA_EINVAL, "bad execution stats arguments");
  const int nl = q->spec.num_leaves;
  for (int t = 0; t < num_trees; ++t) {
    int rc = check_tree(ops, num_ops, tree_root[t], nl);
    if (rc) return rc;
  }
  hipStream_t st = (hipStream_t)stream;
  if (docs_scanned < 0 && !q->scanned_since_fetch) docs_scanned = q->last_matched;
  if (docs_scanned < 0) {  // numDocsScanned of the last scan, from its counter (no fetch since the scan)
    unsigned long long d = 0;
    PA_HIP(hipMemcpyAsync(&d, q->sections.back().ptr, 8, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    docs_scanned = (int64_t)d;
  }
  // the scan's own counts of a two-scan AND (fused statistics)
  std::vector<int64_t> fused;
  if (q->leap_leaf >= 0) {
    fused.resize((size_t)q->nseg * 3);
    int rc = pa_query_leap_counts(q, fused.data(), stream);
    if (rc) return rc;
  }
  std::vector<Plan> plans(q->nseg);
  std::vector<int> state(q->nseg, 0);  // 0: plan, 1: constant known (fused / non-scan), 2: GPU replay, -1: host
  std::vector<std::pair<int, ReplayFlat>> replays;
  std::vector<int64_t> seg_in(q->nseg, 0);
  int64_t non_scan_docs = 0;
  for (int si = 0; si < q->nseg; ++si) {
    const int t = segment_tree[si];
    const int64_t n = q->segs[si]->num_docs;
    if (t == PA_STATS_NON_SCAN) {
      non_scan_docs += n;
      state[si] = 1;
      continue;
    }
    if (t == PA_STATS_HOST) {
      state[si] = -1;
      continue;
    }
    if (t < 0 || t >= num_trees) return fail(PA_EINVAL, "execution stats: segment tree index out of range");
    const int root = tree_root[t];
    const pa_filter_op& r = ops[root];
    if (!fused.empty() && !fused[3 * si + 2] && r.kind == PA_FOP_AND && r.num_children == 2) {
      // AND(Z scan, E scan) counted by the scan: n + |Z & E| + leaps (the leap-frog's reads telescope)
      const pa_filter_op& a = ops[root + 1];
      const pa_filter_op& b = ops[root + 2];
      if (a.kind == PA_FOP_SCAN && b.kind == PA_FOP_SCAN && a.mv_column < 0 && b.mv_column < 0 && a.prog_len == 1 &&
          b.prog_len == 1 && b.prog[0] == q->leap_leaf && a.prog[0] == 1 - q->leap_leaf) {
        seg_in[si] = n + fused[3 * si] + fused[3 * si + 1];
        state[si] = 1;
        continue;
      }
    }
    Ctx x{q, si, ops, num_ops, &plans[si]};
    try {
      seg_in[si] = cost_next(x, root, false);
    } catch (const Unsupported&) {
      // outside the reduction: the iterator tree replayed on the GPU (stat_replay_kernel), else on the host
      plans[si] = Plan{};
      seg_in[si] = 0;
      try {
        Replay R;
        R.root = replay_build(x, root, R);
        replays.push_back({si, replay_flatten(R)});
        state[si] = 2;
      } catch (const Unsupported&) {
        plans[si] = Plan{};
        state[si] = -1;
      }
    }
  }
  // GPU work: leaf bitmaps of the segments with counts or leap-frogs, their element masks, the counts, the leap-frogs
  std::vector<int> leaf_lit(nl, -1);
  for (int l = 0; l < nl; ++l) {
    for (size_t i = 0; i < q->literals.size() && leaf_lit[l] < 0; ++i)
      if (q->literals[i].leaf == l) leaf_lit[l] = (int)i;
  }
  std::map<std::pair<int, std::vector<int32_t>>, int> mask_id;
  std::vector<std::pair<int, std::vector<int32_t>>> masks;
  auto mask_of = [&](int si, const std::vector<int32_t>& p) {
    auto key = std::make_pair(si, p);
    auto it = mask_id.find(key);
    if (it != mask_id.end()) return it->second;
    const int id = (int)masks.size();
    mask_id.emplace(key, id);
    masks.push_back(key);
    return id;
  };
  struct CountReq { int si, mask; int32_t mv; };
  struct LeapReq { int si; const Leap* lp; };
  std::vector<CountReq> creq;
  std::vector<LeapReq> lreq, breq;  // breq: two single-value scans leap-frogged (closed form over label counts)
  std::vector<char> seg_bm(q->nseg, 0);
  for (const auto& rp : replays)
    for (const RNode& nd : rp.second.nodes)
      if (nd.kind == RP_DOCS || nd.kind == RP_SCAN) mask_of(rp.first, nd.prog);
  for (int si = 0; si < q->nseg; ++si) {
    if (state[si] != 0 && state[si] != 2) continue;
    for (const auto& c : plans[si].counts) creq.push_back(CountReq{si, mask_of(si, c.first), c.second});
    for (const Leap& lp : plans[si].leaps) {
      if (lp.el.size() == 2 && !lp.tail && lp.el[0].kind == LF_SCAN && lp.el[1].kind == LF_SCAN && lp.el[0].mv < 0 &&
          lp.el[1].mv < 0 && (int)lp.el[0].prog.size() <= kBitProgMax && (int)lp.el[1].prog.size() <= kBitProgMax) {
        // AndDocIdIterator over two SVScanDocIdIterators reads num_docs + |A & B| + leaps (pa_kernels.hip word_leaps)
        breq.push_back(LeapReq{si, &lp});
        seg_bm[si] = 1;
        continue;
      }
      for (const Elem& e : lp.el) {
        mask_of(si, e.prog);
        for (const Elem& s : e.subs) mask_of(si, s.prog);
      }
      lreq.push_back(LeapReq{si, &lp});
    }
  }
  for (const auto& m : masks) seg_bm[m.first] = 1;
  int gpu_segs = 0;
  if (!masks.empty() || !breq.empty() || !replays.empty()) {
    for (int l = 0; l < nl; ++l)
      if (leaf_lit[l] < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
    std::vector<int64_t> bm_off(q->nseg, -1);
    size_t bm_words = 0;
    for (int si = 0; si < q->nseg; ++si)
      if (seg_bm[si]) {
        bm_off[si] = (int64_t)bm_words;
        bm_words += (size_t)nl * (size_t)leaf_words(q->segs[si]->num_docs);
        ++gpu_segs;
      }
    // the two-scan leap-frogs: pa_bitmap_counts' jobs (programs A, B over the segment's leaf bitmaps)
    std::vector<BitJob> bjobs(breq.size());
    std::vector<int32_t> btok(breq.size() * 2 * kBitProgMax, 0);
    std::vector<size_t> bsc(breq.size());
    size_t bsc_words = 0;
    int64_t bblocks = 0;
    for (size_t r = 0; r < breq.size(); ++r) {
      const Leap& lp = *breq[r].lp;
      const int64_t n = q->segs[breq[r].si]->num_docs, words = leaf_words(n);
      int32_t* t = btok.data() + r * 2 * kBitProgMax;
      const int la = (int)lp.el[0].prog.size(), lb = (int)lp.el[1].prog.size();
      std::copy(lp.el[0].prog.begin(), lp.el[0].prog.end(), t);
      std::copy(lp.el[1].prog.begin(), lp.el[1].prog.end(), t + kBitProgMax);
      bsc[r] = bsc_words;
      bsc_words += (size_t)bit_count_scratch_words(words) + 2;
      bjobs[r] = make_bit_job(nullptr, words, n, bblocks, nullptr, la, lb, nullptr, nullptr);
      renumber_leaves(bjobs[r], t);
      bblocks += bjobs[r].nb;
    }
    std::vector<int64_t> mk_off(masks.size());
    size_t mk_words = 0;
    std::vector<int32_t> toks;
    std::vector<StatMaskJob> mjobs(masks.size());
    int64_t mblocks = 0;
    for (size_t m = 0; m < masks.size(); ++m) {
      const int si = masks[m].first;
      const int64_t words = leaf_words(q->segs[si]->num_docs);
      mk_off[m] = (int64_t)mk_words;
      mk_words += (size_t)words;
      int depth = 0, maxd = 0;
      for (int32_t t : masks[m].second) {
        if (t >= 0) maxd = std::max(maxd, ++depth);
        else if (t != PA_BIT_NOT) --depth;
      }
      if (maxd > kBitProgStack) return fail(PA_EUNSUPPORTED, "execution stats: doc-set program too deep");
      StatMaskJob& j = mjobs[m];
      j = StatMaskJob{};
      j.words = words;
      j.num_docs = q->segs[si]->num_docs;
      j.first_block = mblocks;
      j.tok_off = (int32_t)toks.size();
      j.len = (int32_t)masks[m].second.size();
      toks.insert(toks.end(), masks[m].second.begin(), masks[m].second.end());
      mblocks += stat_mask_blocks(words);
    }
    std::vector<StatCountJob> cjobs(creq.size());
    int64_t cblocks = 0;
    for (size_t r = 0; r < creq.size(); ++r) {
      const int64_t words = leaf_words(q->segs[creq[r].si]->num_docs);
      cjobs[r] = StatCountJob{};
      cjobs[r].words = words;
      cjobs[r].first_block = cblocks;
      cblocks += stat_mask_blocks(words);
    }
    std::vector<LfJob> ljobs(lreq.size());
    int64_t lanes = 0;
    size_t cell_words = 0;
    for (size_t r = 0; r < lreq.size(); ++r) {
      LfJob& j = ljobs[r];
      j = LfJob{};
      const Leap& lp = *lreq[r].lp;
      j.K = (int32_t)lp.el.size();
      j.num_docs = q->segs[lreq[r].si]->num_docs;
      j.nchunks = (j.num_docs + kLfChunkDocs - 1) / kLfChunkDocs;
      int ns = 0;
      for (int e = 0; e < j.K; ++e) {
        j.kind[e] = lp.el[e].kind;
        j.sub_first[e] = ns;
        j.sub_count[e] = (int32_t)lp.el[e].subs.size();
        for (const Elem& s : lp.el[e].subs) j.sub_kind[ns++] = s.kind;
      }
      j.nsub = ns;
      j.cell_words = 4 + 2 * ns;
      j.first_lane = lanes;
      lanes += j.nchunks * (j.K + 1);
      cell_words += (size_t)(j.nchunks * (j.K + 1) * j.cell_words);
    }
    std::vector<LeafJob> leafjobs;
    int64_t lblocks = 0;
    for (int si = 0; si < q->nseg; ++si) {
      if (bm_off[si] < 0 || q->segs[si]->num_docs == 0) continue;
      const int64_t n = q->segs[si]->num_docs, words = leaf_words(n);
      for (int l = 0; l < nl; ++l) {
        leafjobs.push_back(LeafJob{(const DevSeg*)q->dsegs.p + si, nullptr, n, lblocks, leaf_lit[l],
                                   q->literals[leaf_lit[l]].neg ? 1 : 0});
        leafjobs.back().out = (uint32_t*)(intptr_t)(bm_off[si] + (int64_t)l * words);  // (word offset; rebased below)
        lblocks += leaf_bitmap_blocks(n);
      }
    }
    const size_t nres = creq.size() + 3 * lreq.size() + 4 * breq.size() + replays.size();
    const size_t o_bm = 0, o_mk = align256(4 * bm_words), o_cells = o_mk + align256(4 * mk_words),
                 o_res = o_cells + align256(4 * std::max<size_t>(1, cell_words)),
                 o_bsc = o_res + align256(8 * std::max<size_t>(1, nres)),
                 o_bj = o_bsc + align256(4 * std::max<size_t>(1, bsc_words)),
                 o_btok = o_bj + align256(sizeof(BitJob) * std::max<size_t>(1, bjobs.size())),
                 o_btab = o_btok + align256(4 * std::max<size_t>(1, btok.size())),
                 o_mj = o_btab + align256(4 * (size_t)std::max<int64_t>(1, bblocks)),
                 o_cj = o_mj + align256(sizeof(StatMaskJob) * std::max<size_t>(1, mjobs.size())),
                 o_lj = o_cj + align256(sizeof(StatCountJob) * std::max<size_t>(1, cjobs.size())),
                 o_fj = o_lj + align256(sizeof(LfJob) * std::max<size_t>(1, ljobs.size())),
                 o_tok = o_fj + align256(sizeof(LeafJob) * std::max<size_t>(1, leafjobs.size())),
                 o_rp = o_tok + align256(4 * std::max<size_t>(1, toks.size())),
                 total = o_rp + sizeof(RpJob) * std::max<size_t>(1, replays.size());
    if (q->stat_buf.n < total) {
      dev_free(q->stat_buf);
      int rc = dev_alloc(q->stat_buf, total);
      if (rc) return rc;
    }
    char* base = (char*)q->stat_buf.p;
    const uint32_t* bm = (const uint32_t*)(base + o_bm);
    uint32_t* mk = (uint32_t*)(base + o_mk);
    unsigned long long* res = (unsigned long long*)(base + o_res);
    for (size_t m = 0; m < masks.size(); ++m) {
      mjobs[m].bm = bm + bm_off[masks[m].first];
      mjobs[m].out = mk + mk_off[m];
    }
    for (size_t r = 0; r < creq.size(); ++r) {
      cjobs[r].mask = mk + mk_off[creq[r].mask];
      cjobs[r].wt = creq[r].mv >= 0 ? (const int32_t*)q->segs[creq[r].si]->cols.at(creq[r].mv)->mv_off.p : nullptr;
      cjobs[r].out = res + r;
    }
    size_t cell_at = 0;
    for (size_t r = 0; r < lreq.size(); ++r) {
      LfJob& j = ljobs[r];
      const int si = lreq[r].si;
      const Leap& lp = *lreq[r].lp;
      int ns = 0;
      for (int e = 0; e < j.K; ++e) {
        const Elem& el = lp.el[e];
        j.emask[e] = mk + mk_off[mask_id.at(std::make_pair(si, el.prog))];
        j.ewt[e] = el.mv >= 0 ? (const int32_t*)q->segs[si]->cols.at(el.mv)->mv_off.p : nullptr;
        for (const Elem& s : el.subs) {
          j.smask[ns] = mk + mk_off[mask_id.at(std::make_pair(si, s.prog))];
          j.swt[ns] = s.mv >= 0 ? (const int32_t*)q->segs[si]->cols.at(s.mv)->mv_off.p : nullptr;
          ++ns;
        }
      }
      j.cells = (uint32_t*)(base + o_cells) + cell_at;
      cell_at += (size_t)(j.nchunks * (j.K + 1) * j.cell_words);
      j.out = res + creq.size() + 3 * r;
    }
    for (LeafJob& lj : leafjobs) lj.out = (uint32_t*)(base + o_bm) + (intptr_t)lj.out;
    const size_t rres = creq.size() + 3 * lreq.size() + 4 * breq.size();
    std::vector<RpJob> rjobs(replays.size());
    for (size_t r = 0; r < replays.size(); ++r) {
      const int si = replays[r].first;
      const ReplayFlat& F = replays[r].second;
      RpJob& j = rjobs[r];
      std::memset(&j, 0, sizeof(j));
      j.num_docs = q->segs[si]->num_docs;
      j.nnodes = (int32_t)F.nodes.size();
      j.root = 0;
      int nk = 0;
      for (size_t i = 0; i < F.nodes.size(); ++i) {
        const RNode& nd = F.nodes[i];
        RpNode& o = j.node[i];
        o.kind = nd.kind;
        o.depth = F.depth[i];
        o.first = nk;
        o.nchild = (int32_t)nd.kids.size();
        for (int c : nd.kids) j.kids[nk++] = c;
        if (nd.kind == RP_DOCS || nd.kind == RP_SCAN) o.mask = mk + mk_off[mask_id.at(std::make_pair(si, nd.prog))];
        if (nd.mv >= 0) o.wt = (const int32_t*)q->segs[si]->cols.at(nd.mv)->mv_off.p;
      }
      j.out = res + rres + r;
    }
    if (!rjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_rp, rjobs.data(), sizeof(RpJob) * rjobs.size(), hipMemcpyHostToDevice, st));
    const size_t bres = creq.size() + 3 * lreq.size();
    for (size_t r = 0; r < breq.size(); ++r) {
      BitJob& j = bjobs[r];
      j.bm = bm + bm_off[breq[r].si];
      j.tok = (const int32_t*)(base + o_btok) + r * 2 * kBitProgMax;
      j.scratch = (uint32_t*)(base + o_bsc) + bsc[r];
      j.part = (unsigned long long*)(((uintptr_t)(j.scratch + 2 * j.nb) + 7) & ~(uintptr_t)7);
      j.out = res + bres + 4 * r;
    }
    if (!mjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_mj, mjobs.data(), sizeof(StatMaskJob) * mjobs.size(), hipMemcpyHostToDevice, st));
    if (!bjobs.empty()) {
      PA_HIP(hipMemcpyAsync(base + o_bj, bjobs.data(), sizeof(BitJob) * bjobs.size(), hipMemcpyHostToDevice, st));
      PA_HIP(hipMemcpyAsync(base + o_btok, btok.data(), 4 * btok.size(), hipMemcpyHostToDevice, st));
    }
    if (!cjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_cj, cjobs.data(), sizeof(StatCountJob) * cjobs.size(), hipMemcpyHostToDevice, st));
    if (!ljobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_lj, ljobs.data(), sizeof(LfJob) * ljobs.size(), hipMemcpyHostToDevice, st));
    if (!leafjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_fj, leafjobs.data(), sizeof(LeafJob) * leafjobs.size(), hipMemcpyHostToDevice, st));
    if (!toks.empty()) PA_HIP(hipMemcpyAsync(base + o_tok, toks.data(), 4 * toks.size(), hipMemcpyHostToDevice, st));
    PA_HIP(hipMemsetAsync(res, 0, 8 * std::max<size_t>(1, nres), st));
    if (!leafjobs.empty())
      PA_HIP(launch_leaf_bitmaps_batch((const LeafJob*)(base + o_fj), (int)leafjobs.size(), lblocks, st));
    PA_HIP(launch_stat_masks((const StatMaskJob*)(base + o_mj), (int)mjobs.size(), mblocks,
                             (const int32_t*)(base + o_tok), st));
    PA_HIP(launch_stat_counts((const StatCountJob*)(base + o_cj), (int)cjobs.size(), cblocks, st));
    PA_HIP(launch_leapfrogs((const LfJob*)(base + o_lj), (int)ljobs.size(), lanes, st));
    PA_HIP(launch_bit_counts_batch((const BitJob*)(base + o_bj), (int)bjobs.size(), bblocks, true,
                                   (int32_t*)(base + o_btab), st));
    PA_HIP(launch_stat_replay((const RpJob*)(base + o_rp), (int)rjobs.size(), st));
    std::vector<int64_t> h(std::max<size_t>(1, nres));
    PA_HIP(hipMemcpyAsync(h.data(), res, 8 * h.size(), hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    for (size_t r = 0; r < creq.size(); ++r) seg_in[creq[r].si] += h[r];
    for (size_t r = 0; r < lreq.size(); ++r)
      seg_in[lreq[r].si] += h[creq.size() + 3 * r] + (lreq[r].lp->tail ? h[creq.size() + 3 * r + 1] : 0);
    for (size_t r = 0; r < breq.size(); ++r)
      seg_in[breq[r].si] += (int64_t)q->segs[breq[r].si]->num_docs + h[bres + 4 * r + 2] + h[bres + 4 * r + 3];
    for (size_t r = 0; r < replays.size(); ++r) {
      if ((uint64_t)h[rres + r] == ~0ull) return fail(PA_EHIP, "execution stats: iterator replay did not finish");
      seg_in[replays[r].first] += h[rres + r];
    }
  }
  int64_t in_filter = 0;
  for (int si = 0; si < q->nseg; ++si) {
    if (state[si] < 0) seg_in[si] = -1;
    else if (segment_tree[si] == PA_STATS_NON_SCAN) seg_in[si] = 0;
    else in_filter += seg_in[si];
    if (segment_in_filter) segment_in_filter[si] = seg_in[si];
  }
  out[0] = in_filter;
  out[1] = (docs_scanned - non_scan_docs) * (int64_t)projected_columns;
  out[2] = gpu_segs;
  return PA_OK;
}

}  // extern "C"
