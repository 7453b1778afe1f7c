// FAN_FAULT grammar (host-only, no HIP): "site:index:kind[,site:index:kind...]" with kind one of flip, nan,
// delay_ms=<milliseconds>. Parsed completely up front so a malformed rule fails at engine construction, never in
// the middle of a request. Shared with the Python engine's fpga_ai_nic_amd/utils/faults.py.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fan {

struct FaultRule {
  std::string site;
  int64_t index;     // which call of `site` (0-based) the rule fires on
  std::string kind;  // "flip", "nan", "delay_ms" or "drop" (a site that sends: the message is never announced)
  double delay_ms = 0.0;
};

// Throws std::invalid_argument naming the offending rule.
std::vector<FaultRule> parse_fault_spec(const std::string& spec);

}  // namespace fan
