// Host-only self-test of the native ring planner, built with AddressSanitizer + UndefinedBehaviorSanitizer
// ("ASAN builds of the host C++"). Driven by tests/test_native_sanitizers.py.
//
// Checks, for every world 1..9 and blocks 1..3, by simulating all ring positions together:
//   * what position p sends in round j is exactly what its upstream neighbour p-1 receives in round j;
//   * reduce-scatter: every slice is reduced by exactly N contributions and owned by exactly one position,
//     the owner being p-1 (hw/all_reduce.sv:1230);
//   * all-gather: every position ends with every slice, fully reduced;
// and that ring_orders() returns arc-disjoint Hamiltonian cycles (Tillson decomposition).
#include <cstdio>
#include <cstdlib>
#include <set>
#include <utility>
#include <vector>

#include "comm/planner.h"

using namespace fan;

static int failures = 0;
#define EXPECT(c, ...)                                   \
  do {                                                   \
    if (!(c)) {                                          \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                 \
      std::fprintf(stderr, "\n");                        \
      ++failures;                                        \
    }                                                    \
  } while (0)

static void check_plan(int N, int blocks) {
  std::vector<std::vector<RingRound>> plans;
  for (int p = 0; p < N; ++p) plans.push_back(ring_plan(N, p, blocks));
  const size_t rows = plans[0].size();
  for (int p = 0; p < N; ++p) EXPECT(plans[p].size() == rows, "N=%d: rows differ", N);
  const int nsl = N * blocks;
  // contributions[p][slice] = set of ranks whose gradient is inside the partial p holds for `slice`
  std::vector<std::vector<std::set<int>>> partial(N, std::vector<std::set<int>>(nsl));
  std::vector<std::vector<int>> full(N, std::vector<int>(nsl, 0));
  std::vector<int> owners(nsl, -1);
  for (size_t j = 0; j < rows; ++j) {
    std::vector<std::pair<int, std::set<int>>> sent(N, {-1, {}});
    std::vector<int> sent_full(N, 0);
    for (int p = 0; p < N; ++p) {
      const RingRound& r = plans[p][j];
      if (r.send_slice < 0) continue;
      EXPECT(r.send_slice < nsl, "slice out of range");
      std::set<int> c;
      if (r.send_src == kSendLocal) {
        c = {p};
      } else if (r.send_src == kSendReduce) {
        c = partial[p][r.send_slice];
        EXPECT(!c.empty(), "N=%d p=%d row %zu: reduce without a received partial", N, p, j);
        EXPECT(!c.count(p), "N=%d p=%d: own contribution added twice", N, p);
        c.insert(p);
      } else if (r.send_src == kSendForward) {
        EXPECT(full[p][r.send_slice], "N=%d p=%d: forwarding a slice not yet fully reduced", N, p);
        for (int q = 0; q < N; ++q) c.insert(q);
        sent_full[p] = 1;
      }
      if (r.owned >= 0) {
        EXPECT(r.owned == r.send_slice, "owned != send_slice");
        EXPECT((int)c.size() == N, "N=%d p=%d: owned slice has %zu contributions", N, p, c.size());
        EXPECT(owners[r.owned] < 0, "slice %d owned twice", r.owned);
        EXPECT(r.owned % N == (p - 1 + N) % N, "N=%d p=%d owns slice %d (expected position p-1)", N, p, r.owned);
        owners[r.owned] = p;
        full[p][r.owned] = 1;
        sent_full[p] = 1;
      }
      sent[p] = {r.send_slice, c};
    }
    for (int p = 0; p < N; ++p) {
      const RingRound& r = plans[p][j];
      if (r.recv_slice < 0) continue;
      const int up = (p + 1) % N;  // p receives from p+1 (p+1 sends to its downstream p)
      EXPECT(sent[up].first == r.recv_slice, "N=%d row %zu: p=%d expects slice %d, upstream sent %d", N, j, p,
             r.recv_slice, sent[up].first);
      if (r.recv_full) {
        EXPECT((int)sent[up].second.size() == N, "N=%d: recv_full of a partial slice", N);
        full[p][r.recv_slice] = 1;
      } else {
        partial[p][r.recv_slice] = sent[up].second;
      }
    }
  }
  if (N == 1) {
    for (int s = 0; s < nsl; ++s) EXPECT(owners[s] == 0, "N=1: slice %d not owned", s);
    return;
  }
  for (int s = 0; s < nsl; ++s) EXPECT(owners[s] >= 0, "N=%d blocks=%d: slice %d never owned", N, blocks, s);
  for (int p = 0; p < N; ++p)
    for (int s = 0; s < nsl; ++s) EXPECT(full[p][s], "N=%d: position %d misses slice %d", N, p, s);
}

static void check_orders(int N) {
  const auto orders = ring_orders(N, N - 1 > 0 ? N - 1 : 1);
  std::set<std::pair<int, int>> arcs;
  for (const auto& o : orders) {
    EXPECT((int)o.size() == N, "order size");
    std::set<int> seen(o.begin(), o.end());
    EXPECT((int)seen.size() == N, "order is not a permutation");
    if (N < 2) continue;
    for (int i = 0; i < N; ++i) {
      // the data flows position p -> p-1: the directed arc is (o[p], o[p-1])
      const std::pair<int, int> a{o[i], o[(i - 1 + N) % N]};
      EXPECT(!arcs.count(a), "N=%d: arc %d->%d used by two rings", N, a.first, a.second);
      arcs.insert(a);
    }
  }
  if (N == 8) EXPECT(orders.size() == 7, "8 GPUs should give 7 arc-disjoint rings, got %zu", orders.size());
}

// Rings restricted to a link matrix (links[a * N + b]: a can send to b; topology.link_matrix): every returned
// order is a Hamiltonian cycle whose arcs all exist, arc-disjoint across rings; with no usable cycle the planner
// falls back to the identity order.
static void check_links(int N, const std::vector<char>& links, size_t expect_min) {
  const auto orders = ring_orders(N, N - 1 > 0 ? N - 1 : 1, &links);
  EXPECT(!orders.empty(), "N=%d: no order", N);
  std::set<std::pair<int, int>> arcs;
  bool identity_only = orders.size() == 1;
  for (int i = 0; identity_only && i < N; ++i) identity_only = orders[0][i] == i;
  for (const auto& o : orders) {
    EXPECT((int)o.size() == N, "order size");
    std::set<int> seen(o.begin(), o.end());
    EXPECT((int)seen.size() == N, "order is not a permutation");
    if (N < 2 || identity_only) continue;
    for (int i = 0; i < N; ++i) {
      const int from = o[i], to = o[(i - 1 + N) % N];  // data flows position p -> p-1
      EXPECT(links[(size_t)from * N + to], "N=%d: ring uses missing link %d->%d", N, from, to);
      EXPECT(!arcs.count({from, to}), "N=%d: arc %d->%d used twice", N, from, to);
      arcs.insert({from, to});
    }
  }
  EXPECT(orders.size() >= expect_min, "N=%d: %zu rings, expected >= %zu", N, orders.size(), expect_min);
}

int main() {
  for (int N = 2; N <= 9; ++N) {
    std::vector<char> full((size_t)N * N, 1), ring((size_t)N * N, 0), none((size_t)N * N, 0);
    for (int a = 0; a < N; ++a) {
      full[(size_t)a * N + a] = 0;
      ring[(size_t)a * N + (a + 1) % N] = ring[(size_t)((a + 1) % N) * N + a] = 1;  // a physical bidirectional ring
    }
    check_links(N, full, N == 8 ? 7 : 1);
    check_links(N, ring, 1);
    check_links(N, none, 1);  // nothing usable: identity fallback
  }

  for (int N = 1; N <= 9; ++N) {
    for (int b = 1; b <= 3; ++b) check_plan(N, b);
    check_orders(N);
    for (long n : {1L, 255L, 256L, 100000L, 1L << 22}) {
      const RingGeometry g = ring_geometry(n, N, 4096);
      EXPECT(g.slice_elems % 256 == 0 && g.slice_elems <= 4096, "slice");
      EXPECT(g.n_pad == g.blocks * N * g.slice_elems && g.n_pad >= n, "n_pad");
    }
  }
  bool threw = false;
  try {
    ring_geometry(10, 0, 256);
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw, "world 0 must be rejected");
  if (failures) {
    std::printf("FAILED %d\n", failures);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
