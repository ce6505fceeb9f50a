// Segment residency (pa_segment_*): forward indexes, dictionaries and raw columns uploaded once per segment.
#include "pa_host.h"

namespace {
int upload_dict(Column* c, int32_t vtype, int32_t card, const void* dict_values, const int32_t* dict_hashes) {
  c->vtype = vtype;
  c->cardinality = card;
  if (dict_values != nullptr && (vtype == PA_INT || vtype == PA_LONG || vtype == PA_FLOAT || vtype == PA_DOUBLE)) {
    int rc = dev_alloc(c->dict, (size_t)card * 8);
    if (rc) return rc;
    PA_HIP(hipMemcpy(c->dict.p, dict_values, (size_t)card * 8, hipMemcpyHostToDevice));
    c->hvals.assign((const uint64_t*)dict_values, (const uint64_t*)dict_values + card);
    uint64_t hsh = 1469598103934665603ull ^ (uint64_t)card;
    for (uint64_t v : c->hvals) hsh = (hsh ^ v) * 1099511628211ull;
    c->dict_hash = hsh;
    if (vtype == PA_INT || vtype == PA_LONG) {
      const int64_t* v = (const int64_t*)dict_values;
      c->fits_int32 = true;
      for (int32_t i = 0; i < card && c->fits_int32; ++i) c->fits_int32 = v[i] >= INT32_MIN && v[i] <= INT32_MAX;
    }
    // sorted dictionary (the reference's dictionaries always are: SegmentDictionaryCreator sorts the unique values)
    c->dict_sorted = true;
    for (int32_t i = 1; i < card && c->dict_sorted; ++i)
      c->dict_sorted = value_order_key(c->hvals[i - 1], vtype) < value_order_key(c->hvals[i], vtype);
  }
  if (dict_hashes != nullptr) {
    int rc = dev_alloc(c->hashes, (size_t)card * 4);
    if (rc) return rc;
    PA_HIP(hipMemcpy(c->hashes.p, dict_hashes, (size_t)card * 4, hipMemcpyHostToDevice));
  }
  return PA_OK;
}

}  // namespace

extern "C" {

int pa_abi_version(void) { return PA_ABI_VERSION; }

int pa_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pa_set_device(int device) {
  PA_HIP(hipSetDevice(device));
  return PA_OK;
}

const char* pa_last_error(void) { return g_err.c_str(); }

void* pa_host_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<uint64_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) {
    fail(PA_ENOMEM, "hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

void pa_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

pa_segment* pa_segment_create(int32_t num_docs) {
  if (num_docs < 0) {
    fail(PA_EINVAL, "num_docs < 0");
    return nullptr;
  }
  pa_segment* s = new pa_segment();
  s->num_docs = num_docs;
  return s;
}

int pa_segment_add_sv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value, int32_t cardinality,
                                  int32_t value_type, const void* dict_values, const int32_t* dict_hashes) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (num_bits_per_value < 1 || num_bits_per_value > 31) return fail(PA_EINVAL, "num_bits_per_value must be 1..31");
  if (cardinality < 1) return fail(PA_EINVAL, "cardinality < 1");
  if (value_type < PA_INT || value_type > PA_BYTES) return fail(PA_EINVAL, "bad value_type");
  const uint64_t need = ((uint64_t)seg->num_docs * (uint64_t)num_bits_per_value + 7) / 8;
  if (fwd_index_bytes < need) return fail(PA_EINVAL, "forward index shorter than ceil(numDocs*numBits/8)");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  Column* c = new Column();
  c->kind = COL_SV_DICT;
  c->nbits = num_bits_per_value;
  // guard words | whole wave tiles of 64*nb words | guard words
  const int64_t stream_words = wtiles_for(seg->num_docs) * 64 * num_bits_per_value;
  const int64_t total_words = kGuardWords + stream_words + kGuardWords;
  int rc = dev_alloc(c->words, (size_t)total_words * 4);
  if (rc) { delete c; return rc; }
  uint32_t* w = (uint32_t*)c->words.p;
  if (hipMemset(w, 0, (size_t)total_words * 4) != hipSuccess ||
      hipMemcpy(w + kGuardWords, fwd_index, need, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "forward index upload failed");
  }
  if (launch_bswap_words(w + kGuardWords, (int64_t)((need + 3) / 4), nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "bswap kernel failed");
  }
  rc = upload_dict(c, value_type, cardinality, dict_values, dict_hashes);
  if (rc) { delete c; return rc; }
  seg->bytes += c->words.n + c->dict.n + c->hashes.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int pa_segment_add_mv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value, int32_t cardinality,
                                  int64_t total_num_values, int32_t value_type, const void* dict_values,
                                  const int32_t* dict_hashes) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (num_bits_per_value < 1 || num_bits_per_value > 31) return fail(PA_EINVAL, "num_bits_per_value must be 1..31");
  if (cardinality < 1) return fail(PA_EINVAL, "cardinality < 1");
  if (value_type < PA_INT || value_type > PA_BYTES) return fail(PA_EINVAL, "bad value_type");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  const int64_t nd = seg->num_docs;
  if (total_num_values < nd || total_num_values > INT32_MAX)
    return fail(PA_EINVAL, "total_num_values must be in [num_docs, 2^31) (every MV row holds at least one value)");
  // FixedBitMVForwardIndexReader.java:66-79 section sizes: chunk offsets | row-start bitmap | bit-packed values
  int64_t num_chunks = 0, docs_per_chunk = 1;
  if (nd > 0) {
    const float avg = (float)(total_num_values / nd);  // Java: int / int, then widened
    docs_per_chunk = (int64_t)std::ceil((double)(2048.0f / avg));
    num_chunks = (nd + docs_per_chunk - 1) / docs_per_chunk;
  }
  const uint64_t bitmap_bytes = (uint64_t)(total_num_values + 7) / 8;
  const uint64_t raw_bytes = ((uint64_t)total_num_values * (uint64_t)num_bits_per_value + 7) / 8;
  const uint64_t header = (uint64_t)num_chunks * 4;
  if (fwd_index_bytes < header + bitmap_bytes + raw_bytes)
    return fail(PA_EINVAL, "MV forward index shorter than its chunk-offset, bitmap and value sections");
  const uint8_t* bitmap = fwd_index + header;
  const uint8_t* raw = bitmap + bitmap_bytes;
  // row starts: the set bits of the bitmap, in order (the reader's getNextSetBitOffset walk, done once at load)
  std::vector<int32_t> off((size_t)nd + 1);
  int64_t d = 0;
  for (int64_t v = 0; v < total_num_values; ++v) {
    if (bitmap[v >> 3] & (0x80 >> (v & 7))) {
      if (d >= nd) return fail(PA_EINVAL, "MV bitmap has more row starts than documents");
      off[d++] = (int32_t)v;
    }
  }
  if (d != nd || (nd > 0 && off[0] != 0)) return fail(PA_EINVAL, "MV bitmap row starts do not match num_docs");
  off[nd] = (int32_t)total_num_values;
  int32_t max_values = 1;
  for (int64_t i = 0; i < nd; ++i) max_values = std::max(max_values, off[i + 1] - off[i]);
  for (int64_t ch = 0; ch < num_chunks; ++ch) {  // chunk offsets (big-endian int32) must agree with the bitmap
    const uint8_t* p = fwd_index + 4 * ch;
    const int64_t co = ((int64_t)p[0] << 24) | ((int64_t)p[1] << 16) | ((int64_t)p[2] << 8) | (int64_t)p[3];
    if (co != off[ch * docs_per_chunk]) return fail(PA_EINVAL, "MV chunk offsets disagree with the row-start bitmap");
  }
  Column* c = new Column();
  c->kind = COL_MV_DICT;
  c->nbits = num_bits_per_value;
  c->total_values = total_num_values;
  c->max_values = max_values;
  // guard words | value stream padded to whole 64-value steps | guard words (reads stay in bounds)
  const int64_t stream_words = ((total_num_values + 2047) / 2048) * 64 * num_bits_per_value;
  const int64_t total_words = kGuardWords + stream_words + kGuardWords;
  int rc = dev_alloc(c->words, (size_t)total_words * 4);
  if (!rc) rc = dev_alloc(c->mv_off, off.size() * 4);
  if (rc) { delete c; return rc; }
  uint32_t* w = (uint32_t*)c->words.p;
  if (hipMemset(w, 0, (size_t)total_words * 4) != hipSuccess ||
      hipMemcpy(w + kGuardWords, raw, raw_bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->mv_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "MV forward index upload failed");
  }
  if (launch_bswap_words(w + kGuardWords, (int64_t)((raw_bytes + 3) / 4), nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "bswap kernel failed");
  }
  rc = upload_dict(c, value_type, cardinality, dict_values, dict_hashes);
  if (rc) { delete c; return rc; }
  seg->bytes += c->words.n + c->mv_off.n + c->dict.n + c->hashes.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int pa_segment_add_raw_column(pa_segment* seg, int32_t column_id, int32_t value_type, const void* values) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (value_type < PA_INT || value_type > PA_DOUBLE) return fail(PA_EINVAL, "raw columns must be INT/LONG/FLOAT/DOUBLE");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  const size_t esz = (value_type == PA_INT || value_type == PA_FLOAT) ? 4 : 8;
  Column* c = new Column();
  c->kind = COL_SV_RAW;
  c->vtype = value_type;
  c->fits_int32 = value_type == PA_INT;
  const size_t padded = (size_t)wtiles_for(seg->num_docs) * kWTileDocs;
  int rc = dev_alloc(c->raw, padded * esz + 16);
  if (rc) { delete c; return rc; }
  if (hipMemset(c->raw.p, 0, padded * esz + 16) != hipSuccess ||
      hipMemcpy(c->raw.p, values, (size_t)seg->num_docs * esz, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "raw column upload failed");
  }
  if (value_type == PA_LONG) {  // (Pinot's column metadata min/max): int32-range LONG metrics sum in one int64 slot
    const int64_t* v = (const int64_t*)values;
    bool fits = true;
    for (int32_t i = 0; i < seg->num_docs; ++i) fits &= v[i] >= INT32_MIN && v[i] <= INT32_MAX;
    c->fits_int32 = fits;
  }
  seg->bytes += c->raw.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int32_t pa_segment_num_docs(const pa_segment* seg) { return seg ? seg->num_docs : -1; }
uint64_t pa_segment_device_bytes(const pa_segment* seg) { return seg ? seg->bytes : 0; }
void pa_segment_destroy(pa_segment* seg) { delete seg; }

}  // extern "C"
