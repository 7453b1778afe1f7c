// Ring all-reduce schedule planner (native).
//
// Re-expresses the reference NIC's per-block state machine (hw/all_reduce.sv:832-1086;
// SURVEY.md §2.6 / Appendix B) as a list of communication rounds for one ring position:
//   SEND_LOCAL (1) -> REDUCE (N-2) -> REDUCE_OUTPUT (1) -> FORWARD_OUTPUT (N-2) -> OUTPUT,
// with the reference's block-level software pipeline (OUTPUT_SEND: the last all-gather receive of
// block b shares a round with block b+1's SEND_LOCAL). Position p sends to p-1 and receives from p+1
// (readme.pdf p.2 §2.2); inside a block, p reads slices p, p+1, ..., p+N-1 (mod N) (hw/all_reduce.sv:361)
// and owns slice p-1 (hw/all_reduce.sv:1230).
// Unlike the reference (N in 3..6 only, hw/all_reduce.sv:1152), every N >= 1 is supported.
#pragma once
#include <cstdint>
#include <vector>

namespace fan {

enum RingSendSrc : int32_t {
  kSendNone = -1,
  kSendLocal = 0,    // encode(local[slice])
  kSendReduce = 1,   // encode(decode(recv_prev) + local[slice])
  kSendForward = 2,  // forward the fully reduced slice received in the previous round (no re-encode)
};

struct RingRound {
  int32_t send_slice;  // global slice id (block * N + j) or -1
  int32_t send_src;    // RingSendSrc
  int32_t recv_slice;  // global slice id arriving this round or -1
  int32_t recv_full;   // 1 if the arriving slice is fully reduced (all-gather phase)
  int32_t owned;       // slice whose full sum this position produces this round (== send_slice) or -1
};

struct RingGeometry {
  int64_t n;            // valid elements
  int64_t slice_elems;  // S (multiple of the granule, 256 by default)
  int64_t blocks;       // B
  int64_t n_pad;        // B * N * S
};

// granule: the slice is a multiple of it (256: one wire shard; 256 * P: P sub-shards for a streamed ring hop)
RingGeometry ring_geometry(int64_t n, int world, int64_t max_slice_elems, int64_t granule = 256);
std::vector<RingRound> ring_plan(int world, int position, int64_t blocks);

// Arc-disjoint directed Hamiltonian cycles of the link digraph on `world` vertices (up to world-1 rings; fewer
// when no decomposition exists, e.g. world 4 and 6 on a complete graph). `links` (row-major world x world,
// links[a * world + b] != 0: rank a can send to rank b over a direct link; nullptr: complete graph, the 8-GPU
// fully connected xGMI node) restricts the rings to physical links — the reference builds its single ring from
// the physical Ethernet wiring the same way (sw/setup_route.sh:12-40). With no Hamiltonian cycle over the links
// the identity order is returned (the transport then routes the missing hops).
std::vector<std::vector<int>> ring_orders(int world, int max_rings, const std::vector<char>* links = nullptr);

}  // namespace fan
