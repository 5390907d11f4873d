// Host-side TFRecord framing for the dataset path (datasets/ljspeech/dataset.py:96-112 reads
// tf.data.TFRecordDataset files; preprocess/ljspeech.py:23-45 + utils/tfrecord.py:46-49 write
// them).  A TFRecord is  uint64 length | uint32 masked_crc32c(length) | data |
// uint32 masked_crc32c(data), little endian; masked(c) = ((c >> 15) | (c << 17)) + 0xa282ead8.
// CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), slicing-by-8 tables.  No device code.
#include "sat_common.h"

namespace {

struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFFu];
  }
};

const Crc32cTables& tables() {
  static const Crc32cTables tb;   // immutable after first use (C++11 thread-safe init)
  return tb;
}

}  // namespace

// crc32c of n bytes continuing from `crc` (0 for a fresh checksum)
extern "C" uint32_t sat_crc32c(const void* data, int64_t n, uint32_t crc) {
  const auto& T = tables().t;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  while (n > 0 && (reinterpret_cast<uintptr_t>(p) & 7u)) {
    c = (c >> 8) ^ T[0][(c ^ *p++) & 0xFFu];
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    const uint32_t lo = static_cast<uint32_t>(w) ^ c, hi = static_cast<uint32_t>(w >> 32);
    c = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
        T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n-- > 0) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xFFu];
  return ~c;
}

extern "C" uint32_t sat_tfrecord_masked_crc(const void* data, int64_t n) {
  const uint32_t c = sat_crc32c(data, n, 0u);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// Frame one record: out must hold n + 16 bytes.  Returns the framed size.
extern "C" int64_t sat_tfrecord_frame(const void* data, int64_t n, void* out) {
  uint8_t* o = static_cast<uint8_t*>(out);
  const uint64_t len = static_cast<uint64_t>(n);
  memcpy(o, &len, 8);
  const uint32_t lc = sat_tfrecord_masked_crc(o, 8);
  memcpy(o + 8, &lc, 4);
  memcpy(o + 12, data, static_cast<size_t>(n));
  const uint32_t dc = sat_tfrecord_masked_crc(data, n);
  memcpy(o + 12 + n, &dc, 4);
  return n + 16;
}

// Split a buffer of concatenated records: writes up to `cap` (offset, length) pairs of the
// payloads into `spans` and returns the record count, or a negative SAT_ERR_* code on a
// truncated buffer or a checksum mismatch (verify != 0).
extern "C" int64_t sat_tfrecord_index(const void* buf, int64_t n, int32_t verify, int64_t* spans,
                                      int64_t cap) {
  const uint8_t* b = static_cast<const uint8_t*>(buf);
  int64_t pos = 0, count = 0;
  while (pos < n) {
    if (n - pos < 12) { ::sat::set_error("sat_tfrecord_index: truncated record header"); return SAT_ERR_ARGUMENT; }
    uint64_t len;
    uint32_t lc;
    memcpy(&len, b + pos, 8);
    memcpy(&lc, b + pos + 8, 4);
    if (verify && lc != sat_tfrecord_masked_crc(b + pos, 8)) {
      ::sat::set_error("sat_tfrecord_index: length checksum mismatch");
      return SAT_ERR_ARGUMENT;
    }
    if (len > static_cast<uint64_t>(n - pos - 12) || n - pos - 12 - static_cast<int64_t>(len) < 4) {
      ::sat::set_error("sat_tfrecord_index: truncated record payload");
      return SAT_ERR_ARGUMENT;
    }
    const int64_t off = pos + 12;
    if (verify) {
      uint32_t dc;
      memcpy(&dc, b + off + len, 4);
      if (dc != sat_tfrecord_masked_crc(b + off, static_cast<int64_t>(len))) {
        ::sat::set_error("sat_tfrecord_index: data checksum mismatch");
        return SAT_ERR_ARGUMENT;
      }
    }
    if (count < cap) { spans[2 * count] = off; spans[2 * count + 1] = static_cast<int64_t>(len); }
    ++count;
    pos = off + static_cast<int64_t>(len) + 4;
  }
  return count;
}
