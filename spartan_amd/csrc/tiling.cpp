// Min-cost tiling solver behind the AutomaticTiling pass -- host C++, linked
// into libspx.so and exported through the C ABI (include/spx.h:
// spx_mincost_tiling).  No device code.
//
// Restates the choice procedure of spartan/expr/tiling.cc
// (find_mincost_tiling :31-92, driven by mincost_tiling :94-132) for the cost
// graph AutomaticTiling builds (spartan/expr/optimize.py:454-890).  Nodes are
// (expression, tiling) pairs, node 0 is the source and node t the sink; an
// edge u -> v of cost c means "v consumes u, moving c elements"; a split pair
// {a, b} holds the row / column alternatives of one expression, of which one
// is chosen.  From the source, every out-edge of a node must be satisfied;
// when a node reaches both halves of a split pair, both sub-problems are
// solved on copies of the chosen set and the cheaper is kept -- a tie is put
// back behind the node's remaining out-edges, and resolved towards the second
// half once none remain.  Out-edges are visited most-recently-added first,
// the order of the reference's head-inserted edge lists, since the greedy
// choice depends on it.
//
// The graphs are small (a few nodes per expression): recursive search over
// per-node adjacency vectors, no fixed-size global tables.
#include "../../include/spx.h"

#include <cstdint>
#include <deque>
#include <unordered_map>
#include <vector>

namespace {

constexpr int64_t kUnreachable = 1000000000;  // cost of a half made unreachable by an earlier choice

struct TilingGraph {
  struct Arc {
    int to;
    int64_t cost;
  };
  std::vector<std::vector<Arc>> out;  // per node, visiting order (newest first)
  std::unordered_map<int, int> partner;
  std::vector<int64_t> dist;

  int64_t solve(int s, std::vector<uint8_t>& chosen) {
    const std::vector<Arc>& arcs = out[s];
    int64_t total = 0;
    std::deque<int> todo;
    for (int i = 0; i < (int)arcs.size(); ++i) todo.push_back(i);
    int remaining = (int)todo.size();
    while (!todo.empty()) {
      const int ai = todo.front();
      todo.pop_front();
      --remaining;
      const int v = arcs[ai].to;
      const auto pit = partner.find(v);
      if (pit == partner.end()) {  // an ordinary consumer: always taken
        if (!chosen[v]) {
          dist[v] = solve(v, chosen);
          total += dist[v];
          chosen[v] = 1;
        }
        total += arcs[ai].cost;
        continue;
      }
      const int w = pit->second;
      int aj = -1;  // the partner's arc further down s's list, if any
      for (int k = ai + 1; k < (int)arcs.size(); ++k)
        if (arcs[k].to == w) {
          aj = k;
          break;
        }
      if (aj < 0) {  // s reaches one half only
        if (chosen[v] || chosen[w]) {
          total += chosen[v] ? arcs[ai].cost : kUnreachable;
        } else {
          dist[v] = solve(v, chosen);
          total += dist[v] + arcs[ai].cost;
          chosen[v] = 1;
        }
        continue;
      }
      for (auto it = todo.begin(); it != todo.end(); ++it)
        if (*it == aj) {
          todo.erase(it);
          break;
        }
      --remaining;  // counted as taken even when already gone (a repeated arc)
      if (chosen[v] || chosen[w]) {
        total += chosen[v] ? arcs[ai].cost : arcs[aj].cost;
        continue;
      }
      std::vector<uint8_t> pick_v(chosen), pick_w(chosen);
      dist[v] = solve(v, pick_v);
      dist[w] = solve(w, pick_w);
      const int64_t cv = dist[v] + arcs[ai].cost, cw = dist[w] + arcs[aj].cost;
      if (cv == cw && remaining > 0) {  // undecided: revisit after the other arcs
        todo.push_back(ai);
        todo.push_back(aj);
      } else if (cv < cw) {
        total += cv;
        chosen.swap(pick_v);
        chosen[v] = 1;
      } else {
        total += cw;
        chosen.swap(pick_w);
        chosen[w] = 1;
      }
    }
    return total;
  }
};

}  // namespace

extern "C" int spx_mincost_tiling(int32_t t, int64_t n_edges, const int32_t* eu, const int32_t* ev,
                                  const int64_t* ecost, int64_t n_split, const int32_t* su, const int32_t* sv,
                                  uint8_t* chosen, int64_t* total_cost) {
  if (t < 1 || n_edges < 0 || n_split < 0 || !chosen) return -1;
  if ((n_edges > 0 && (!eu || !ev || !ecost)) || (n_split > 0 && (!su || !sv))) return -1;
  TilingGraph g;
  g.out.assign((size_t)t + 1, {});
  g.dist.assign((size_t)t + 1, 0);
  for (int64_t i = 0; i < n_edges; ++i) {
    if (eu[i] < 0 || eu[i] > t || ev[i] < 0 || ev[i] > t) return -1;
    g.out[eu[i]].push_back({ev[i], ecost[i]});
  }
  for (auto& arcs : g.out) {  // newest first
    for (size_t i = 0, j = arcs.size(); i + 1 < j; ++i, --j) std::swap(arcs[i], arcs[j - 1]);
  }
  for (int64_t i = 0; i < n_split; ++i) {
    if (su[i] < 0 || su[i] > t || sv[i] < 0 || sv[i] > t) return -1;
    g.partner[su[i]] = sv[i];
    g.partner[sv[i]] = su[i];
  }
  std::vector<uint8_t> sel((size_t)t + 1, 0);
  const int64_t cost = g.solve(0, sel);
  for (int i = 0; i < t; ++i) chosen[i] = sel[i];
  if (total_cost) *total_cost = cost;
  return 0;
}
