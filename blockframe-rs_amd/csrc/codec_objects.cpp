// codec_objects.cpp — bfrs_encoder / bfrs_decoder: the stateful surface of
// reed_solomon_simd::ReedSolomonEncoder / ReedSolomonDecoder (3.x) as the
// reference uses it (src/chunker/generate.rs:37-49,84-96;
// src/filestore/recovery.rs:58-69,152-170; src/filestore/health.rs:733-752).
//
// Shards added from host memory are copied straight into device memory (the
// crate likewise copies each added shard into its work area); encode()/decode()
// run the HIP pass and bring the results back to host buffers owned by the
// object, valid until the next call on it.
#include <sstream>

#include "runtime.hpp"

using namespace bfrs;

namespace {

struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

size_t stride_of(size_t shard_bytes) { return (shard_bytes + 255) / 256 * 256; }

int shard_size_error(size_t expected, size_t got) {
  std::ostringstream os;
  os << "different shard size: expected " << expected << " bytes, got " << got << " bytes";
  return set_error(BFRS_E_DIFFERENT_SHARD_SIZE, os.str());
}

}  // namespace

struct bfrs_encoder {
  bfrs_ctx *ctx;
  size_t k, m, shard_bytes;
  size_t received = 0;
  bool encoded = false;
  DevBuf dev;                              // (k + m) shard slots
  std::vector<std::vector<uint8_t>> recovery;
};

struct bfrs_decoder {
  bfrs_ctx *ctx;
  size_t k, m, shard_bytes;
  std::vector<uint8_t> orig_present, rec_present;
  bool decoded = false;
  DevBuf dev;                              // (k + m) shard slots
  std::vector<std::vector<uint8_t>> restored;  // index by original; empty = not restored
};

extern "C" {

int bfrs_encoder_new(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes, bfrs_encoder **out) {
  BFRS_API_BEGIN
  if (!ctx || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_encoder_new: NULL argument");
  *out = nullptr;
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  auto *e = new (std::nothrow) bfrs_encoder{ctx, k, m, shard_bytes};
  if (!e) return set_error(BFRS_E_NOMEM, "encoder allocation failed");
  hipError_t he = hipSetDevice(ctx->impl.device);
  if (he == hipSuccess) he = hipMalloc(&e->dev.p, stride_of(shard_bytes) * (k + m));
  if (he != hipSuccess) {
    delete e;
    return hip_error(he, "bfrs_encoder_new: hipMalloc");
  }
  *out = e;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_encoder_add_original_shard(bfrs_encoder *e, const uint8_t *shard, size_t len) {
  BFRS_API_BEGIN
  if (!e || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_original_shard: NULL argument");
  if (e->encoded) {  // the crate resets an encoder once its result is released
    e->encoded = false;
    e->received = 0;
  }
  if (e->received >= e->k) {
    std::ostringstream os;
    os << "too many original shards: got more than original_count (" << e->k << ") shards";
    return set_error(BFRS_E_TOO_MANY_ORIGINAL_SHARDS, os.str());
  }
  if (len != e->shard_bytes) return shard_size_error(e->shard_bytes, len);
  hipError_t he = hipSetDevice(e->ctx->impl.device);
  if (he == hipSuccess)
    he = hipMemcpy(static_cast<uint8_t *>(e->dev.p) + e->received * stride_of(e->shard_bytes),
                   shard, len, hipMemcpyHostToDevice);
  if (he != hipSuccess) return hip_error(he, "add_original_shard: hipMemcpy");
  ++e->received;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_encoder_encode(bfrs_encoder *e) {
  BFRS_API_BEGIN
  if (!e) return set_error(BFRS_E_INVALID_ARGUMENT, "encode: NULL encoder");
  if (e->received < e->k || e->encoded) {
    std::ostringstream os;
    os << "too few original shards: got " << (e->encoded ? 0 : e->received)
       << " shards while original_count is " << e->k;
    return set_error(BFRS_E_TOO_FEW_ORIGINAL_SHARDS, os.str());
  }
  const size_t st = stride_of(e->shard_bytes);
  auto *d = static_cast<uint8_t *>(e->dev.p);
  std::vector<const uint8_t *> din(e->k);
  std::vector<uint8_t *> dout(e->m);
  for (size_t i = 0; i < e->k; ++i) din[i] = d + i * st;
  for (size_t j = 0; j < e->m; ++j) dout[j] = d + (e->k + j) * st;
  uint32_t kk = uint32_t(e->k);
  int rc = encode_batch_on(e->ctx, 1, &kk, e->m, e->shard_bytes, din.data(), dout.data(),
                           e->ctx->impl.stream);
  if (rc) return rc;
  e->recovery.assign(e->m, std::vector<uint8_t>(e->shard_bytes));
  Context &c = e->ctx->impl;
  for (size_t j = 0; j < e->m; ++j) {
    hipError_t he = hipMemcpyAsync(e->recovery[j].data(), dout[j], e->shard_bytes,
                                   hipMemcpyDeviceToHost, c.stream);
    if (he != hipSuccess) return hip_error(he, "encode: D2H");
  }
  hipError_t he = hipStreamSynchronize(c.stream);
  if (he != hipSuccess) return hip_error(he, "encode: sync");
  e->encoded = true;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_encoder_recovery(bfrs_encoder *e, size_t index, const uint8_t **data, size_t *len) {
  BFRS_API_BEGIN
  if (!e || !data || !len) return set_error(BFRS_E_INVALID_ARGUMENT, "recovery: NULL argument");
  if (!e->encoded || index >= e->recovery.size()) {
    std::ostringstream os;
    os << "invalid recovery shard index: " << index << " >= recovery_count " << e->m;
    return set_error(BFRS_E_INVALID_RECOVERY_SHARD_INDEX, os.str());
  }
  *data = e->recovery[index].data();
  *len = e->recovery[index].size();
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_encoder_free(bfrs_encoder *e) { delete e; }

int bfrs_decoder_new(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes, bfrs_decoder **out) {
  BFRS_API_BEGIN
  if (!ctx || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_decoder_new: NULL argument");
  *out = nullptr;
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  auto *d = new (std::nothrow) bfrs_decoder{ctx, k, m, shard_bytes};
  if (!d) return set_error(BFRS_E_NOMEM, "decoder allocation failed");
  d->orig_present.assign(k, 0);
  d->rec_present.assign(m, 0);
  hipError_t he = hipSetDevice(ctx->impl.device);
  if (he == hipSuccess) he = hipMalloc(&d->dev.p, stride_of(shard_bytes) * (k + m));
  if (he != hipSuccess) {
    delete d;
    return hip_error(he, "bfrs_decoder_new: hipMalloc");
  }
  *out = d;
  return BFRS_OK;
  BFRS_API_END
}

static void decoder_reset_if_done(bfrs_decoder *d) {
  if (d->decoded) {
    d->decoded = false;
    d->restored.clear();
    std::fill(d->orig_present.begin(), d->orig_present.end(), 0);
    std::fill(d->rec_present.begin(), d->rec_present.end(), 0);
  }
}

int bfrs_decoder_add_original_shard(bfrs_decoder *d, size_t index, const uint8_t *shard,
                                    size_t len) {
  BFRS_API_BEGIN
  if (!d || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_original_shard: NULL argument");
  decoder_reset_if_done(d);
  if (index >= d->k) {
    std::ostringstream os;
    os << "invalid original shard index: " << index << " >= original_count " << d->k;
    return set_error(BFRS_E_INVALID_ORIGINAL_SHARD_INDEX, os.str());
  }
  if (d->orig_present[index]) {
    std::ostringstream os;
    os << "duplicate original shard index: " << index;
    return set_error(BFRS_E_DUPLICATE_ORIGINAL_SHARD_INDEX, os.str());
  }
  if (len != d->shard_bytes) return shard_size_error(d->shard_bytes, len);
  hipError_t he = hipSetDevice(d->ctx->impl.device);
  if (he == hipSuccess)
    he = hipMemcpy(static_cast<uint8_t *>(d->dev.p) + index * stride_of(d->shard_bytes), shard,
                   len, hipMemcpyHostToDevice);
  if (he != hipSuccess) return hip_error(he, "add_original_shard: hipMemcpy");
  d->orig_present[index] = 1;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_add_recovery_shard(bfrs_decoder *d, size_t index, const uint8_t *shard,
                                    size_t len) {
  BFRS_API_BEGIN
  if (!d || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_recovery_shard: NULL argument");
  decoder_reset_if_done(d);
  if (index >= d->m) {
    std::ostringstream os;
    os << "invalid recovery shard index: " << index << " >= recovery_count " << d->m;
    return set_error(BFRS_E_INVALID_RECOVERY_SHARD_INDEX, os.str());
  }
  if (d->rec_present[index]) {
    std::ostringstream os;
    os << "duplicate recovery shard index: " << index;
    return set_error(BFRS_E_DUPLICATE_RECOVERY_SHARD_INDEX, os.str());
  }
  if (len != d->shard_bytes) return shard_size_error(d->shard_bytes, len);
  hipError_t he = hipSetDevice(d->ctx->impl.device);
  if (he == hipSuccess)
    he = hipMemcpy(static_cast<uint8_t *>(d->dev.p) + (d->k + index) * stride_of(d->shard_bytes),
                   shard, len, hipMemcpyHostToDevice);
  if (he != hipSuccess) return hip_error(he, "add_recovery_shard: hipMemcpy");
  d->rec_present[index] = 1;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_decode(bfrs_decoder *d) {
  BFRS_API_BEGIN
  if (!d) return set_error(BFRS_E_INVALID_ARGUMENT, "decode: NULL decoder");
  size_t orig_recv = 0, rec_recv = 0;
  for (uint8_t b : d->orig_present) orig_recv += b;
  for (uint8_t b : d->rec_present) rec_recv += b;
  if (orig_recv + rec_recv < d->k) {
    std::ostringstream os;
    os << "not enough shards: " << orig_recv << " original + " << rec_recv << " recovery < "
       << d->k << " original_count";
    return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
  }
  d->restored.assign(d->k, {});
  d->decoded = true;
  if (orig_recv == d->k) return BFRS_OK;

  const size_t st = stride_of(d->shard_bytes);
  auto *base = static_cast<uint8_t *>(d->dev.p);
  // Restored shards are written over the erased originals' own slots.
  std::vector<const uint8_t *> dorig(d->k), drec(d->m);
  std::vector<uint8_t *> drest(d->k, nullptr);
  for (size_t i = 0; i < d->k; ++i) {
    if (d->orig_present[i])
      dorig[i] = base + i * st;
    else
      drest[i] = base + i * st;
  }
  for (size_t j = 0; j < d->m; ++j)
    if (d->rec_present[j]) drec[j] = base + (d->k + j) * st;
  uint32_t kk = uint32_t(d->k);
  int rc = decode_batch_on(d->ctx, 1, &kk, d->m, d->shard_bytes, dorig.data(), drec.data(),
                           drest.data(), d->ctx->impl.stream);
  if (rc) return rc;
  Context &c = d->ctx->impl;
  for (size_t i = 0; i < d->k; ++i)
    if (!d->orig_present[i]) {
      d->restored[i].resize(d->shard_bytes);
      hipError_t he = hipMemcpyAsync(d->restored[i].data(), drest[i], d->shard_bytes,
                                     hipMemcpyDeviceToHost, c.stream);
      if (he != hipSuccess) return hip_error(he, "decode: D2H");
    }
  hipError_t he = hipStreamSynchronize(c.stream);
  if (he != hipSuccess) return hip_error(he, "decode: sync");
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_restored_original(bfrs_decoder *d, size_t index, const uint8_t **data,
                                   size_t *len) {
  BFRS_API_BEGIN
  if (!d || !data || !len)
    return set_error(BFRS_E_INVALID_ARGUMENT, "restored_original: NULL argument");
  *data = nullptr;
  *len = 0;
  if (!d->decoded || index >= d->restored.size() || d->restored[index].empty())
    return set_error(BFRS_E_NOT_RESTORED, "original shard was not restored");
  *data = d->restored[index].data();
  *len = d->restored[index].size();
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_decoder_free(bfrs_decoder *d) { delete d; }

}  // extern "C"
