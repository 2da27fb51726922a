// cooc_codec.cpp — the ItemCooccurrences wire format (host only, no device calls).
//
// ItemCooccurrences.Serializer (ItemCooccurrences.java:113-147) writes, per record,
//   output.writeInt(item, true)      Kryo variable-length int, optimizePositive
//   output.writeShort(increment)     2 bytes, big-endian
//   output.writeInt(size', true)     size' = size (k == -1) or size - 1 (slot k skipped, :124-131)
//   size' x output.writeInt(other, true)
// and reads it back with k == -1 (:135-146).  The Kryo primitives are those of Kryo 2.24.0, the
// version Flink 1.3.2 ships (a Maven dependency, not vendored under /root/reference): a varint is
// the int's 32 bits in 7-bit groups, least significant first, bit 7 set on every byte but the last,
// at most 5 bytes (Output.writeVarInt / Input.readVarInt); a short is (v >>> 8, v) as two bytes
// (Output.writeShort / Input.readShort).  A negative int takes 5 bytes with optimizePositive.
//
// A mixed deployment that keeps the Java emitter (NonSampled...java:138-151) and offloads the
// reducer decodes the records it receives with cooc_records_decode; the reverse direction (device
// results consumed by an unchanged Java reducer) encodes with cooc_records_encode.
#include <cstdint>
#include <cstring>

#include "../../include/cooc.h"

namespace {

inline int64_t varint_size(uint32_t v) {
  int64_t n = 1;
  while (v >>= 7) n++;
  return n;
}

inline uint8_t *put_varint(uint8_t *p, uint32_t v) {  // Output.writeVarInt(v, true)
  while (v >= 0x80) {
    *p++ = uint8_t(v & 0x7F) | 0x80;
    v >>= 7;
  }
  *p++ = uint8_t(v);
  return p;
}

// Input.readVarInt(true): false on a truncated stream.  The fifth byte contributes its low 4 bits
// (<< 28); Kryo does not check the rest, and neither does this reader.
inline bool get_varint(const uint8_t *&p, const uint8_t *end, int32_t *out) {
  uint32_t r = 0;
  for (int i = 0; i < 5; i++) {
    if (p >= end) return false;
    const uint8_t b = *p++;
    r |= uint32_t(b & 0x7F) << (7 * i);
    if (!(b & 0x80) || i == 4) {
      *out = int32_t(r);
      return true;
    }
  }
  return false;
}

}  // namespace

extern "C" {

COOC_API int cooc_records_encode(int64_t n_records, const int32_t *items, const int16_t *increments, const int32_t *ks,
                                 const int64_t *rec_ptr, const int32_t *others, uint8_t *out, int64_t out_cap,
                                 int64_t *n_bytes) {
  if (n_records < 0 || !n_bytes || (n_records > 0 && (!items || !increments || !rec_ptr))) return COOC_ERR_ARG;
  int64_t total = 0;
  for (int64_t r = 0; r < n_records; r++) {
    const int64_t lo = rec_ptr[r], hi = rec_ptr[r + 1];
    if (hi < lo || (hi > lo && !others)) return COOC_ERR_ARG;
    const int64_t size = hi - lo, k = ks ? ks[r] : -1;
    if (k != -1 && (k < 0 || k >= size)) return COOC_ERR_ARG;  // the writer would skip nothing / overrun
    total += varint_size(uint32_t(items[r])) + 2 + varint_size(uint32_t(k == -1 ? size : size - 1));
    for (int64_t i = 0; i < size; i++)
      if (i != k) total += varint_size(uint32_t(others[lo + i]));
  }
  *n_bytes = total;
  if (!out) return COOC_OK;  // size query (two-phase protocol)
  if (out_cap < total) return COOC_ERR_ARG;
  uint8_t *p = out;
  for (int64_t r = 0; r < n_records; r++) {
    const int64_t lo = rec_ptr[r], size = rec_ptr[r + 1] - lo, k = ks ? ks[r] : -1;
    p = put_varint(p, uint32_t(items[r]));
    const uint16_t inc = uint16_t(increments[r]);
    *p++ = uint8_t(inc >> 8);  // writeShort: high byte first
    *p++ = uint8_t(inc);
    p = put_varint(p, uint32_t(k == -1 ? size : size - 1));
    for (int64_t i = 0; i < size; i++)
      if (i != k) p = put_varint(p, uint32_t(others[lo + i]));
  }
  return COOC_OK;
}

COOC_API int cooc_records_decode(const uint8_t *bytes, int64_t n_bytes, int64_t *n_records, int64_t *n_others,
                                 int32_t *items, int16_t *increments, int64_t *rec_ptr, int32_t *others) {
  if (n_bytes < 0 || !n_records || !n_others || (n_bytes > 0 && !bytes)) return COOC_ERR_ARG;
  const bool fill = items || increments || rec_ptr || others;
  const uint8_t *p = bytes, *end = bytes + n_bytes;
  int64_t r = 0, o = 0;
  if (fill && rec_ptr) rec_ptr[0] = 0;
  while (p < end) {
    int32_t item, size;
    if (!get_varint(p, end, &item) || end - p < 2) return COOC_ERR_ARG;  // truncated record
    const int16_t inc = int16_t(uint16_t(p[0]) << 8 | uint16_t(p[1]));  // readShort
    p += 2;
    if (!get_varint(p, end, &size)) return COOC_ERR_ARG;
    if (size < 0) return COOC_ERR_ARG;  // new int[size] throws NegativeArraySizeException (:139)
    if (fill) {
      if (items) items[r] = item;
      if (increments) increments[r] = inc;
    }
    for (int32_t i = 0; i < size; i++) {
      int32_t v;
      if (!get_varint(p, end, &v)) return COOC_ERR_ARG;
      if (fill && others) others[o] = v;
      o++;
    }
    r++;
    if (fill && rec_ptr) rec_ptr[r] = o;
  }
  *n_records = r;
  *n_others = o;
  return COOC_OK;
}

}  // extern "C"
