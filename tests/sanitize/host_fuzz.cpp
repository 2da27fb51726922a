// host_fuzz.cpp — the library's host-only parsers under AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/test_sanitize_cpu.py builds this with g++ -fsanitize=address,undefined against the sources in
// flink-cooccurrence_amd/csrc and runs it).  Untrusted bytes reach two entry points: the Kryo record
// decoder (cooc_records_decode, ItemCooccurrences.java:135-146) and the text splitter
// (cooc_parse_interactions, FlinkCooccurrences.java:207-229).  Each is driven through its two-phase
// protocol with random valid inputs (round trips must hold), every truncation of them, bit-flipped and
// random byte strings (must fail cleanly or decode within the sizes the sizing pass reported), and the
// encoder with random records.  Any out-of-bounds access or undefined operation aborts the run.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../include/cooc.h"

namespace {

int fail(const char *what, int64_t i) {
  std::fprintf(stderr, "host_fuzz: %s (case %lld)\n", what, (long long)i);
  return 1;
}

// decode through the two-phase protocol into buffers of exactly the reported sizes
int decode_exact(const std::vector<uint8_t> &b, std::vector<int32_t> *items, std::vector<int16_t> *inc,
                 std::vector<int64_t> *rp, std::vector<int32_t> *others) {
  int64_t nr = 0, no = 0;
  const uint8_t *p = b.empty() ? nullptr : b.data();
  int st = cooc_records_decode(p, int64_t(b.size()), &nr, &no, nullptr, nullptr, nullptr, nullptr);
  if (st != COOC_OK) return st;
  items->assign(size_t(nr), 0);
  inc->assign(size_t(nr), 0);
  rp->assign(size_t(nr) + 1, 0);
  others->assign(size_t(no), 0);
  return cooc_records_decode(p, int64_t(b.size()), &nr, &no, items->data(), inc->data(), rp->data(), others->data());
}

}  // namespace

int main() {
  std::mt19937_64 rng(20261017);
  auto u = [&](int64_t lo, int64_t hi) { return lo + int64_t(rng() % uint64_t(hi - lo + 1)); };
  // ---- records: random round trips, every truncation, bit flips
  for (int c = 0; c < 300; c++) {
    const int64_t n = u(0, 40);
    std::vector<int32_t> items(static_cast<size_t>(n)), ks(static_cast<size_t>(n)), others;
    std::vector<int16_t> incs(static_cast<size_t>(n));
    std::vector<int64_t> rp(1, 0);
    for (int64_t r = 0; r < n; r++) {
      items[size_t(r)] = int32_t(uint32_t(rng()));
      incs[size_t(r)] = int16_t(uint16_t(rng()));
      const int64_t len = u(0, 30);
      for (int64_t j = 0; j < len; j++) others.push_back(u(0, 3) ? int32_t(u(0, 300)) : int32_t(uint32_t(rng())));
      rp.push_back(int64_t(others.size()));
      ks[size_t(r)] = (len > 0 && u(0, 2) == 0) ? int32_t(u(0, len - 1)) : -1;
    }
    int64_t nb = 0;
    const int32_t *kp = (c & 1) ? ks.data() : nullptr;
    if (cooc_records_encode(n, items.data(), incs.data(), kp, rp.data(), others.data(), nullptr, 0, &nb) != COOC_OK)
      return fail("encode sizing", c);
    std::vector<uint8_t> buf(static_cast<size_t>(nb));
    if (cooc_records_encode(n, items.data(), incs.data(), kp, rp.data(), others.data(), buf.data(), nb, &nb) != COOC_OK)
      return fail("encode", c);
    if (nb > 0 && cooc_records_encode(n, items.data(), incs.data(), kp, rp.data(), others.data(), buf.data(), nb - 1,
                                      &nb) == COOC_OK)
      return fail("encode into a short buffer accepted", c);
    std::vector<int32_t> di, dot;
    std::vector<int16_t> dinc;
    std::vector<int64_t> drp;
    if (decode_exact(buf, &di, &dinc, &drp, &dot) != COOC_OK) return fail("decode of an encoding", c);
    if (int64_t(di.size()) != n) return fail("round trip record count", c);
    for (int64_t r = 0; r < n; r++)
      if (di[size_t(r)] != items[size_t(r)] || dinc[size_t(r)] != incs[size_t(r)]) return fail("round trip record", c);
    for (size_t cut = 0; cut < buf.size(); cut += 1 + buf.size() / 64) {  // truncations: clean failure or fewer records
      std::vector<uint8_t> t(buf.begin(), buf.begin() + long(cut));
      (void)decode_exact(t, &di, &dinc, &drp, &dot);
    }
    for (int f = 0; f < 8 && !buf.empty(); f++) {  // bit flips
      std::vector<uint8_t> t = buf;
      t[size_t(u(0, int64_t(t.size()) - 1))] ^= uint8_t(1u << u(0, 7));
      (void)decode_exact(t, &di, &dinc, &drp, &dot);
    }
  }
  for (int c = 0; c < 2000; c++) {  // random byte strings
    std::vector<uint8_t> t(static_cast<size_t>(u(0, 64)));
    for (auto &x : t) x = uint8_t(rng());
    std::vector<int32_t> di, dot;
    std::vector<int16_t> dinc;
    std::vector<int64_t> drp;
    (void)decode_exact(t, &di, &dinc, &drp, &dot);
  }
  // ---- text: valid lines round trip; random text fails cleanly or parses within the counted records
  const char *alphabet = "0123456789,-+\r\n \tx";
  for (int c = 0; c < 3000; c++) {
    std::string s;
    const int64_t lines = u(0, 20);
    std::vector<int64_t> want;
    const bool valid = c % 2 == 0;
    for (int64_t l = 0; l < lines; l++) {
      if (valid) {
        const int64_t a = int32_t(uint32_t(rng())), b = int32_t(uint32_t(rng())), t = int64_t(rng() >> 1);
        s += std::to_string(a) + "," + std::to_string(b) + "," + std::to_string(t) + (u(0, 3) ? "\n" : "\r\n");
        want.push_back(a);
      } else {
        const int64_t len = u(0, 30);
        for (int64_t k = 0; k < len; k++) s += alphabet[u(0, 17)];
        s += "\n";
      }
    }
    if (valid && !s.empty() && u(0, 1)) s.pop_back();  // a last line without '\n'
    int64_t n = 0, bad = 0;
    if (cooc_parse_interactions(s.data(), int64_t(s.size()), 0, nullptr, nullptr, nullptr, &n, &bad) != COOC_OK)
      return fail("text sizing", c);
    std::vector<int32_t> us(static_cast<size_t>(n) + 1), its(static_cast<size_t>(n) + 1);
    std::vector<int64_t> ts(static_cast<size_t>(n) + 1);
    const int st = cooc_parse_interactions(s.data(), int64_t(s.size()), n, us.data(), its.data(), ts.data(), &n, &bad);
    if (valid) {
      if (st != COOC_OK || n != int64_t(want.size())) return fail("valid text", c);
      for (size_t k = 0; k < want.size(); k++)
        if (us[k] != want[k]) return fail("valid text user", c);
    } else if (st != COOC_OK && (bad < 0 || bad > n)) {
      return fail("bad_line outside the records", c);
    }
    if (n > 0 && cooc_parse_interactions(s.data(), int64_t(s.size()), n - 1, us.data(), its.data(), ts.data(), &n,
                                         &bad) == COOC_OK)
      return fail("a capacity below the record count accepted", c);
  }
  std::printf("host_fuzz ok\n");
  return 0;
}
