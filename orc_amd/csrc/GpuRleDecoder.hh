// C++ adapter: the reference's RleDecoder / ByteRleDecoder surface over the
// liborcgpu C ABI (include/orcg.h). Header-only; host code only.
//
// Reference interfaces mirrored (apache/orc):
//   class RleDecoder { seek(PositionProvider&); skip(uint64_t);
//                      next(int64_t*|int32_t*|int16_t*, uint64_t, const char*); }
//       c++/src/RLE.hh:109-141, created by createRleDecoder (RLE.hh:163,
//       RLE.cc:48-60)
//   class ByteRleDecoder { seek; skip; next(char*, uint64_t, char*); }
//       c++/src/ByteRLE.hh:71-93, factories :114, :126
//   orc::ParseError / orc::InvalidArgument (c++/include/orc/Exceptions.hh)
//
// Inside the reference build these classes derive from orc::RleDecoder and
// orc::ByteRleDecoder and are returned by createRleDecoder /
// createBooleanRleDecoder (INTEGRATION.md shows the patch). Standalone (this
// repo's tests) they use the stand-in base classes below, which have the
// reference's exact member signatures.
#pragma once

#include <cstdint>
#include <list>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orcg.h"

namespace orcg {
namespace cxx {

// orc::ParseError / orc::InvalidArgument stand-ins (same what() strings).
class ParseError : public std::runtime_error {
 public:
  explicit ParseError(const std::string& m) : std::runtime_error(m) {}
};
class InvalidArgument : public std::runtime_error {
 public:
  explicit InvalidArgument(const std::string& m) : std::runtime_error(m) {}
};
class DeviceError : public std::runtime_error {
 public:
  explicit DeviceError(const std::string& m) : std::runtime_error(m) {}
};

inline void throwOnError(int rc, const char* msg) {
  switch (rc) {
    case ORCG_OK:
      return;
    case ORCG_PARSE_ERROR:
      throw ParseError(msg);
    case ORCG_INVALID_ARGUMENT:
      throw InvalidArgument(msg);
    default:
      throw DeviceError(msg);
  }
}

// orc::PositionProvider (c++/src/io/InputStream.hh:36-44): a cursor over
// row-index positions.
class PositionProvider {
 public:
  explicit PositionProvider(const std::list<uint64_t>& positions)
      : positions_(positions.begin(), positions.end()) {}
  uint64_t next() { return positions_.at(pos_++); }
  uint64_t current() { return positions_.at(pos_); }
  // the positions still to be consumed (what a decoder's seek() takes)
  std::vector<uint64_t> remaining() const {
    return std::vector<uint64_t>(positions_.begin() + pos_, positions_.end());
  }
  void consume(size_t n) { pos_ += n; }

 private:
  std::vector<uint64_t> positions_;
  size_t pos_ = 0;
};

// RAII device context (one per reader thread).
class Context {
 public:
  explicit Context(int device = 0) {
    if (orcg_ctx_create(device, &ctx_) != ORCG_OK)
      throw DeviceError("no usable HIP device; the orc_amd decoder has no CPU fallback");
  }
  ~Context() { orcg_ctx_destroy(ctx_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  orcg_ctx* get() const { return ctx_; }

 private:
  orcg_ctx* ctx_ = nullptr;
};

// Stand-in bases with the reference's member signatures.
class RleDecoder {
 public:
  virtual ~RleDecoder() = default;
  virtual void seek(PositionProvider&) = 0;
  virtual void skip(uint64_t numValues) = 0;
  virtual void next(int64_t* data, uint64_t numValues, const char* notNull) = 0;
  virtual void next(int32_t* data, uint64_t numValues, const char* notNull) = 0;
  virtual void next(int16_t* data, uint64_t numValues, const char* notNull) = 0;
};

class ByteRleDecoder {
 public:
  virtual ~ByteRleDecoder() = default;
  virtual void seek(PositionProvider&) = 0;
  virtual void skip(uint64_t numValues) = 0;
  virtual void next(char* data, uint64_t numValues, char* notNull) = 0;
};

// GPU RLEv2 decoder: the stream is bulk-decoded on the device on creation.
// (The status is read before the message: the message buffer is only valid
// after the call that set it.)
class GpuRleDecoderV2 : public RleDecoder {
 public:
  GpuRleDecoderV2(Context& ctx, const uint8_t* data, uint64_t len, bool isSigned) {
    const int rc = orcg_rle_decoder_create(ctx.get(), data, len, isSigned ? 1 : 0, 2, &dec_);
    throwOnError(rc, orcg_ctx_last_error(ctx.get()));
  }
  ~GpuRleDecoderV2() override { orcg_rle_decoder_destroy(dec_); }

  // uncompressed stream position: {byte offset, values to skip}
  void seek(PositionProvider& location) override {
    std::vector<uint64_t> p = location.remaining();
    if (p.size() > 2) p.resize(2);
    check(orcg_rle_decoder_seek(dec_, p.data(), p.size()));
    location.consume(p.size());
  }
  void skip(uint64_t n) override { check(orcg_rle_decoder_skip(dec_, n)); }
  void next(int64_t* d, uint64_t n, const char* nn) override { check(orcg_rle_decoder_next_i64(dec_, d, n, nn)); }
  void next(int32_t* d, uint64_t n, const char* nn) override { check(orcg_rle_decoder_next_i32(dec_, d, n, nn)); }
  void next(int16_t* d, uint64_t n, const char* nn) override { check(orcg_rle_decoder_next_i16(dec_, d, n, nn)); }

 private:
  void check(int rc) const { throwOnError(rc, orcg_rle_decoder_last_error(dec_)); }
  orcg_rle_decoder* dec_ = nullptr;
};

// GPU byte / boolean RLE decoder.
class GpuByteRleDecoder : public ByteRleDecoder {
 public:
  GpuByteRleDecoder(Context& ctx, const uint8_t* data, uint64_t len, bool boolean) : boolean_(boolean) {
    const int rc = orcg_byte_rle_decoder_create(ctx.get(), data, len, boolean ? 1 : 0, &dec_);
    throwOnError(rc, orcg_ctx_last_error(ctx.get()));
  }
  ~GpuByteRleDecoder() override { orcg_byte_rle_decoder_destroy(dec_); }
  void seek(PositionProvider& location) override {
    std::vector<uint64_t> p = location.remaining();
    const size_t k = boolean_ ? 3 : 2;
    if (p.size() > k) p.resize(k);
    check(orcg_byte_rle_decoder_seek(dec_, p.data(), p.size()));
    location.consume(p.size());
  }
  void skip(uint64_t n) override { check(orcg_byte_rle_decoder_skip(dec_, n)); }
  void next(char* d, uint64_t n, char* nn) override { check(orcg_byte_rle_decoder_next(dec_, d, n, nn)); }

 private:
  void check(int rc) const { throwOnError(rc, orcg_byte_rle_decoder_last_error(dec_)); }
  orcg_byte_rle_decoder* dec_ = nullptr;
  bool boolean_;
};

// createRleDecoder / createByteRleDecoder / createBooleanRleDecoder shapes.
inline std::unique_ptr<RleDecoder> createGpuRleDecoder(Context& ctx, const uint8_t* data, uint64_t len,
                                                       bool isSigned) {
  return std::make_unique<GpuRleDecoderV2>(ctx, data, len, isSigned);
}
inline std::unique_ptr<ByteRleDecoder> createGpuByteRleDecoder(Context& ctx, const uint8_t* data, uint64_t len) {
  return std::make_unique<GpuByteRleDecoder>(ctx, data, len, false);
}
inline std::unique_ptr<ByteRleDecoder> createGpuBooleanRleDecoder(Context& ctx, const uint8_t* data, uint64_t len) {
  return std::make_unique<GpuByteRleDecoder>(ctx, data, len, true);
}

}  // namespace cxx
}  // namespace orcg
