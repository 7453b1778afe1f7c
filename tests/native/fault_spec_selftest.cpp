// Host-only self-test of the FAN_FAULT grammar parser (csrc/comm/fault_spec.cpp), built with AddressSanitizer +
// UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py: valid specs parse to the expected rules, every
// malformed one throws std::invalid_argument (never crashes, never reads out of bounds, never overflows).
#include <cstdio>
#include <stdexcept>
#include <string>

#include "comm/fault_spec.h"

using namespace fan;

static int failures = 0;
#define EXPECT(c, ...)                                          \
  do {                                                          \
    if (!(c)) {                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
      ++failures;                                               \
    }                                                           \
  } while (0)

static bool throws(const std::string& s) {
  try {
    parse_fault_spec(s);
  } catch (const std::invalid_argument&) {
    return true;
  }
  return false;
}

int main() {
  auto r = parse_fault_spec("mesh_pack:0:flip,mesh_reduce:12:nan,,ring_send:3:delay_ms=2.5");
  EXPECT(r.size() == 3, "3 rules, got %zu", r.size());
  if (r.size() == 3) {
    EXPECT(r[0].site == "mesh_pack" && r[0].index == 0 && r[0].kind == "flip", "rule 0");
    EXPECT(r[1].site == "mesh_reduce" && r[1].index == 12 && r[1].kind == "nan", "rule 1");
    EXPECT(r[2].site == "ring_send" && r[2].index == 3 && r[2].kind == "delay_ms" && r[2].delay_ms == 2.5, "rule 2");
  }
  EXPECT(parse_fault_spec("").empty(), "empty spec");
  {  // 'drop' only where a message is announced (the P2P rounds' flag writes)
    auto d = parse_fault_spec("p2p_publish:1:drop");
    EXPECT(d.size() == 1 && d[0].kind == "drop" && d[0].index == 1, "p2p_publish drop");
  }
  EXPECT(parse_fault_spec(",,,").empty(), "only separators");
  EXPECT(parse_fault_spec("a:999999999999999999:flip")[0].index == 999999999999999999LL, "18-digit index");
  for (const char* s : {"x", "a:1", "a:1:", ":1:flip", "a::flip", "a:-1:flip", "a:1x:flip", "a:1:boom",
                        "a:1:delay_ms=", "a:1:delay_ms=abc", "a:1:delay_ms=-3", "a:1:delay_ms=1e400",
                        "a:1:delay_ms=nan", "a:1:delay_ms=5ms", "a:9999999999999999999:flip", "a:1:flip,b",
                        "a:1:delay_ms=inf", "a:1:FLIP", "\\x01:\\x02:\\x03", "ring_send:0:drop",
                        "mesh_pack:2:drop"})
    EXPECT(throws(s), "'%s' must be rejected", s);
  // every prefix of a long valid spec parses or throws cleanly (bounds / UB under the sanitizers)
  const std::string longspec = "mesh_pack:0:flip,mesh_reduce:7:nan,ring_send:42:delay_ms=0.125";
  for (size_t n = 0; n <= longspec.size(); ++n) {
    try {
      parse_fault_spec(longspec.substr(0, n));
    } catch (const std::invalid_argument&) {
    }
  }
  if (failures) {
    std::printf("FAILED %d\n", failures);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
