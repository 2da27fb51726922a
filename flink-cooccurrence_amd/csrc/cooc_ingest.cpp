// cooc_ingest.cpp — the job's text source in front of the operator (host only, no device calls).
//
// FlinkCooccurrences.java:55-61 reads the input with a TextInputFormat (UnsplittableTextInputFormat.java):
// records are the '\n'-delimited lines, a '\r' before the '\n' is dropped, a last line without '\n'
// is a record, and an empty string after the final '\n' is not.  InteractionLineSplitter (:207-219)
// maps a line with line.split(",") to Tuple3(Integer.valueOf(f0), Integer.valueOf(f1),
// Long.valueOf(f2)): fields after the third are ignored, fewer than three fail, and every field must
// be an optional sign followed by decimal digits in range (no spaces) or the job fails with
// NumberFormatException.  The timestamps feed an AscendingTimestampExtractor (:221-229), whose
// watermark is the largest timestamp seen minus 1.
#include <cstdint>

#include "../../include/cooc.h"

namespace {

// Integer.valueOf / Long.valueOf over [p, e): optional '+'/'-', >= 1 ASCII digit, in range.
template <class T>
bool parse_int(const char *p, const char *e, int64_t lo, int64_t hi, T *out) {
  if (p == e) return false;
  bool neg = false;
  if (*p == '+' || *p == '-') {
    neg = *p == '-';
    if (++p == e) return false;
  }
  // accumulate the magnitude as unsigned: |Long.MIN_VALUE| fits in uint64
  const uint64_t lim = neg ? uint64_t(-(lo + 1)) + 1 : uint64_t(hi);
  uint64_t v = 0;
  for (; p < e; p++) {
    if (*p < '0' || *p > '9') return false;
    const uint64_t d = uint64_t(*p - '0');
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? T(int64_t(0) - int64_t(v - 1) - 1) : T(v);
  return true;
}

// One line [p, e) -> (user, item, ts).  String.split(",") drops trailing empty fields only, so a
// line "1,2,3,,," still has three fields and "1,,3" has an empty (invalid) second field.
bool parse_line(const char *p, const char *e, int32_t *u, int32_t *it, int64_t *ts) {
  const char *f[4] = {p, nullptr, nullptr, nullptr};
  int nf = 1;
  for (const char *q = p; q < e && nf < 4; q++)
    if (*q == ',') f[nf++] = q + 1;
  if (nf < 3) return false;  // split[2] -> ArrayIndexOutOfBoundsException
  const char *e0 = f[1] - 1, *e1 = f[2] - 1;
  const char *e2 = nf > 3 ? f[3] - 1 : e;
  return parse_int(f[0], e0, INT32_MIN, INT32_MAX, u) && parse_int(f[1], e1, INT32_MIN, INT32_MAX, it) &&
         parse_int(f[2], e2, INT64_MIN, INT64_MAX, ts);
}

}  // namespace

extern "C" {

COOC_API int cooc_parse_interactions(const char *text, int64_t n_bytes, int64_t cap, int32_t *users, int32_t *items,
                                     int64_t *ts, int64_t *n_records, int64_t *bad_line) {
  if (n_bytes < 0 || !n_records || (n_bytes > 0 && !text)) return COOC_ERR_ARG;
  const bool fill = users && items && ts;
  const char *p = text, *end = text + n_bytes;
  int64_t n = 0;
  if (bad_line) *bad_line = -1;
  while (p < end) {
    const char *nl = p;
    while (nl < end && *nl != '\n') nl++;
    const char *e = nl;
    if (e > p && e[-1] == '\r') e--;  // TextInputFormat drops the '\r' of "\r\n"
    if (fill) {
      if (n >= cap) return COOC_ERR_ARG;
      if (!parse_line(p, e, users + n, items + n, ts + n)) {
        if (bad_line) *bad_line = n;
        return COOC_ERR_ARG;
      }
    }
    n++;
    p = nl < end ? nl + 1 : end;
  }
  *n_records = n;
  return COOC_OK;
}

}  // extern "C"
