// Ring schedule planner + multi-ring (arc-disjoint Hamiltonian cycle) builder. See planner.h.
#include "comm/planner.h"

#include <algorithm>
#include <functional>
#include <stdexcept>

namespace fan {

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

RingGeometry ring_geometry(int64_t n, int world, int64_t max_slice_elems, int64_t granule) {
  if (world < 1) throw std::invalid_argument("world must be >= 1");
  if (granule < 256 || granule % 256) throw std::invalid_argument("granule must be a multiple of 256");
  if (max_slice_elems < granule) max_slice_elems = granule;
  max_slice_elems = max_slice_elems / granule * granule;
  RingGeometry g;
  g.n = n;
  const int64_t nn = std::max<int64_t>(n, 1);
  g.blocks = cdiv(nn, (int64_t)world * max_slice_elems);
  g.slice_elems = cdiv(cdiv(nn, (int64_t)world * g.blocks), granule) * granule;
  g.n_pad = g.blocks * world * g.slice_elems;
  return g;
}

std::vector<RingRound> ring_plan(int N, int p, int64_t blocks) {
  if (N < 1 || p < 0 || p >= N) throw std::invalid_argument("bad ring position");
  std::vector<RingRound> out;
  auto mod = [N](int64_t x) { return (int32_t)(((x % N) + N) % N); };
  for (int64_t b = 0; b < blocks; ++b) {
    const int32_t base = (int32_t)(b * N);
    if (N == 1) {
      out.push_back({base, kSendLocal, -1, 0, base});
      continue;
    }
    // round 0: SEND_LOCAL; the partner (up = p+1) sends its local slice p+1 in the same round.
    out.push_back({base + mod(p), kSendLocal, base + mod(p + 1), 0, -1});
    // rounds 1..N-2: REDUCE (recv partial p+k+1, send partial p+k)
    for (int k = 1; k <= N - 2; ++k) out.push_back({base + mod(p + k), kSendReduce, base + mod(p + k + 1), 0, -1});
    // round N-1: REDUCE_OUTPUT (this position's slice p-1 is now fully reduced: send + keep);
    //            receives the up position's fully reduced slice p.
    out.push_back({base + mod(p - 1), kSendReduce, base + mod(p), 1, base + mod(p - 1)});
    // rounds N..2N-3: FORWARD_OUTPUT (forward the full slice received last round, receive the next)
    for (int i = 1; i <= N - 2; ++i) out.push_back({base + mod(p + i - 1), kSendForward, base + mod(p + i), 1, -1});
  }
  return out;
}

std::vector<std::vector<int>> ring_orders(int N, int max_rings, const std::vector<char>* links) {
  std::vector<std::vector<int>> best;
  if (N <= 1) return {{0}};
  if (links && (int64_t)links->size() != (int64_t)N * N)
    throw std::invalid_argument("ring_orders: links must be world x world");
  // path arc u -> v carries data v -> u (position p sends to p - 1): it needs the link v -> u
  auto link = [&](int u, int v) { return links == nullptr || (*links)[(size_t)v * N + u] != 0; };
  if (N == 2) return {{0, 1}};
  const int limit = std::max(1, std::min(max_rings, N - 1));
  for (int R = limit; R >= 1; --R) {
    std::vector<std::vector<char>> used(N, std::vector<char>(N, 0));
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) used[i][j] = i == j || !link(i, j);
    std::vector<std::vector<int>> cycles;
    long budget = 2000000;  // bounded search (N <= 16 in practice)
    std::function<bool(int)> find_cycle = [&](int k) -> bool {
      std::vector<int> path{0};
      std::vector<char> in(N, 0);
      in[0] = 1;
      std::function<bool()> dfs = [&]() -> bool {
        if (--budget < 0) return false;
        if ((int)path.size() == N) {
          const int last = path.back();
          if (used[last][0]) return false;
          used[last][0] = 1;
          cycles.push_back(path);
          if (k + 1 == R || find_cycle(k + 1)) return true;
          cycles.pop_back();
          used[last][0] = 0;
          return false;
        }
        const int u = path.back();
        for (int v = 0; v < N; ++v) {
          if (in[v] || used[u][v]) continue;
          used[u][v] = 1;
          in[v] = 1;
          path.push_back(v);
          if (dfs()) return true;
          path.pop_back();
          in[v] = 0;
          used[u][v] = 0;
        }
        return false;
      };
      return dfs();
    };
    if (find_cycle(0)) return cycles;
  }
  std::vector<int> id(N);
  for (int i = 0; i < N; ++i) id[i] = i;
  return {id};
}

}  // namespace fan
