#include "comm/fault_spec.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <stdexcept>

namespace fan {

static void bad(const std::string& item, const std::string& why) {
  throw std::invalid_argument("FAN_FAULT: " + why + " in rule '" + item + "' (expected site:index:kind)");
}

std::vector<FaultRule> parse_fault_spec(const std::string& spec) {
  std::vector<FaultRule> out;
  size_t pos = 0;
  while (pos <= spec.size()) {
    size_t end = spec.find(',', pos);
    if (end == std::string::npos) end = spec.size();
    const std::string item = spec.substr(pos, end - pos);
    pos = end + 1;
    if (item.empty()) continue;
    const size_t a = item.find(':');
    const size_t b = a == std::string::npos ? std::string::npos : item.find(':', a + 1);
    if (a == std::string::npos || b == std::string::npos) bad(item, "missing ':'");
    FaultRule r;
    r.site = item.substr(0, a);
    if (r.site.empty()) bad(item, "empty site");
    const std::string idx = item.substr(a + 1, b - a - 1);
    if (idx.empty() || idx.size() > 18 || idx.find_first_not_of("0123456789") != std::string::npos)
      bad(item, "index must be a non-negative integer");
    r.index = std::strtoll(idx.c_str(), nullptr, 10);
    r.kind = item.substr(b + 1);
    if (r.kind.rfind("delay_ms=", 0) == 0) {
      const std::string v = r.kind.substr(9);
      char* e = nullptr;
      errno = 0;
      const double ms = v.empty() ? -1.0 : std::strtod(v.c_str(), &e);
      if (v.empty() || errno != 0 || e != v.c_str() + v.size() || !std::isfinite(ms) || ms < 0.0 || ms > 3.6e6)
        bad(item, "delay_ms needs a number of milliseconds in [0, 3.6e6]");
      r.kind = "delay_ms";
      r.delay_ms = ms;
    } else if (r.kind == "drop") {
      // only a sending site can lose its announcement (engine.cpp: the P2P rounds' flag writes); at a corrupting
      // site 'drop' would silently do nothing
      if (r.site != "p2p_publish") bad(item, "kind 'drop' applies to site 'p2p_publish' only");
    } else if (r.kind != "flip" && r.kind != "nan") {
      bad(item, "unknown fault kind '" + r.kind + "'");
    }
    out.push_back(r);
  }
  return out;
}

}  // namespace fan
