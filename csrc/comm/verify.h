// Debug verification + fault injection for the native engine's messages.
//
// Verify mode (FAN_VERIFY=1): every message row a rank puts on the fabric gets a tag computed on the GPU —
// {Fletcher-style word sums s1 = sum w_i, s2 = sum (i+1) w_i (mod 2^32), request sequence number, row bytes} —
// and the tags travel with the payload (a second, 16-byte-per-row exchange of the same collective). The receiver
// recomputes the tags of what arrived and a compare kernel records the FIRST mismatch (corrupted payload, or a
// sequence number from another request = a dropped / reordered message) in a device error block, which the host
// reads after the request completes and raises with the site, row and values. Non-blocking on the GPU; the host
// check is in synchronize(). The reference has nothing of the kind: its testbench cannot even check the
// compressed path (readme.pdf p.5), and a lost request hangs forever (hw/README:3-4).
//
// Fault injection (FAN_FAULT="site:index:kind[,...]", test-only; the same grammar as the Python engine's
// fpga_ai_nic_amd/utils/faults.py): sites mesh_pack (the packed shards before the all-to-all), mesh_reduce (the
// owner's reduced shard before the all-gather), ring_send (one ring message); kinds flip (xor the first byte),
// nan (last byte = 0xFF: an exponent of 255), delay_ms=<ms> (the issuing thread stalls the stream's progress);
// site p2p_publish (the ready flags of one direct P2P round) with kind drop: the round is never announced.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "comm/fault_spec.h"
#include "common/hip_common.h"

namespace fan {

struct VerifyError {  // device error block (first mismatch wins)
  uint32_t flag;      // 0 clean, 1 recorded
  uint32_t kind;      // 1 checksum mismatch, 2 sequence mismatch
  uint32_t site;      // caller-defined site id
  uint32_t row;       // row (peer / slice) index of the mismatch
  uint32_t exp_s1, got_s1, exp_seq, got_seq;
};

// tags[r] = {s1, s2, seq, row_bytes} of rows[r] (row_bytes % 16 == 0), rows at row_stride bytes apart.
void launch_msg_tags(const uint8_t* rows, size_t row_bytes, size_t row_stride, int nrows, uint32_t seq, uint32_t* tags,
                     hipStream_t s);
// Recompute the tags of received rows into `scratch` and compare with `recv_tags` (+ expected sequence number);
// the first mismatch goes to `err` with the given site id and row index base.
void launch_msg_verify(const uint8_t* rows, size_t row_bytes, size_t row_stride, int nrows, const uint32_t* recv_tags,
                       uint32_t expect_seq, uint32_t* scratch, VerifyError* err, uint32_t site, uint32_t row_base,
                       hipStream_t s);
// Fault injection: p[0] ^= 0xFF (flip) or p[bytes - 1] = 0xFF (nan).
void launch_fault_byte(uint8_t* p, size_t bytes, int kind, hipStream_t s);


class FaultInjector {
 public:
  FaultInjector();  // from FAN_FAULT
  explicit FaultInjector(const std::string& spec);
  bool active() const { return !rules_.empty(); }
  // apply the rules matching the next call of `site` to buf[0, bytes) on stream s
  void maybe_corrupt(const std::string& site, uint8_t* buf, size_t bytes, hipStream_t s);
  // true when a "drop" rule matches the next call of `site` (the caller then skips the send it guards: a lost
  // message, so the peers' waits never complete — what a dead link looks like; test-only)
  bool maybe_drop(const std::string& site);

 private:
  std::vector<FaultRule> rules_;
  std::map<std::string, int64_t> counts_;
};

}  // namespace fan
