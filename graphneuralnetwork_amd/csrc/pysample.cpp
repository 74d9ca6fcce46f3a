// pysample.cpp -- bit-exact host restatement of the reference GraphSAGE sampler.
//
// Replaces get_layer_adj_nodes (GraphSAGE/data_utils.py:82-124), the index-map half of
// collate_fn (:127-162), and the adj_lists construction of read_pubmed_data (:29-37).
//
// The reference draws from CPython's global `random` (MT19937) and iterates Python
// sets, so its index maps depend on
//   * the Mersenne-Twister stream and how random.sample / random.choices consume it
//     (CPython 3.10 Lib/random.py: sample :438-497, choices :506-519,
//     _randbelow_with_getrandbits :239-249; _randommodule.c genrand_uint32 /
//     getrandbits / random_random), and
//   * the slot order of CPython's open-addressing set table (Objects/setobject.c:
//     set_add_entry with 9 linear probes then perturbed probing, set_insert_clean,
//     set_table_resize, set_merge -- including the re-layout that
//     `layer_nodes.union(...)` does when its copy lands in a differently sized table).
// Both are restated here; the state is CPython's own (random.getstate()[1]: 624 words +
// position), read before and written back after, so a call leaves the Python
// generator exactly where the reference would.  This is sequential host work (one MT
// stream, one set); the GPU sampler (sample.hip) is the throughput path.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/gnn_mi355x.h"

namespace gnn {
namespace {

// ---------------------------------------------------------------- MT19937 (CPython)
struct Mt {
  uint32_t mt[624];
  int index;

  uint32_t next() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    if (index >= 624) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < 624 - 397; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      index = 0;
    }
    uint32_t y = mt[index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // random.random(): 53-bit double from two words
  double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  // random._randbelow(n) for 0 < n < 2^32 (getrandbits(k) = word >> (32 - k), k <= 32)
  int64_t randbelow(int64_t n) {
    if (n <= 0) return 0;
    int k = 0;
    for (uint64_t v = static_cast<uint64_t>(n); v; v >>= 1) ++k;
    uint32_t r = next() >> (32 - k);
    while (r >= static_cast<uint64_t>(n)) r = next() >> (32 - k);
    return r;
  }
};

// ---------------------------------------------------------------- CPython set of ints
// Keys are non-negative ints < 2^61 - 1, whose hash is the value itself; there are no
// deletions, so no dummy entries and fill == used throughout.
constexpr int64_t kEmpty = -1;
constexpr size_t kMinSize = 8;
constexpr size_t kLinearProbes = 9;
constexpr int kPerturbShift = 5;

struct PySet {
  std::vector<int64_t> table;
  size_t mask = kMinSize - 1;
  size_t used = 0;

  PySet() : table(kMinSize, kEmpty) {}

  void clear() {
    table.assign(kMinSize, kEmpty);
    mask = kMinSize - 1;
    used = 0;
  }

  static void insert_clean(std::vector<int64_t>& t, size_t m, int64_t key) {
    size_t perturb = static_cast<size_t>(key);
    size_t i = static_cast<size_t>(key) & m;
    for (;;) {
      if (t[i] == kEmpty) { t[i] = key; return; }
      if (i + kLinearProbes <= m) {
        for (size_t j = 1; j <= kLinearProbes; ++j) {
          if (t[i + j] == kEmpty) { t[i + j] = key; return; }
        }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & m;
    }
  }

  // set_table_resize(so, minused): re-insert the old slots in order into a fresh table
  void resize(size_t minused) {
    size_t newsize = kMinSize;
    while (newsize <= minused) newsize <<= 1;
    std::vector<int64_t> fresh(newsize, kEmpty);
    for (int64_t k : table)
      if (k != kEmpty) insert_clean(fresh, newsize - 1, k);
    table.swap(fresh);
    mask = newsize - 1;
  }

  void found_unused(size_t i, int64_t key) {
    table[i] = key;
    ++used;
    if (used * 5 < mask * 3) return;
    resize(used > 50000 ? used * 2 : used * 4);
  }

  // set_add_entry for an int key
  void add(int64_t key) {
    size_t m = mask;
    size_t i = static_cast<size_t>(key) & m;
    if (table[i] == kEmpty) return found_unused(i, key);
    size_t perturb = static_cast<size_t>(key);
    for (;;) {
      if (table[i] == key) return;
      if (i + kLinearProbes <= m) {
        for (size_t j = 1; j <= kLinearProbes; ++j) {
          const int64_t e = table[i + j];
          if (e == kEmpty) return found_unused(i + j, key);
          if (e == key) return;
        }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & m;
      if (table[i] == kEmpty) return found_unused(i, key);
    }
  }

  // set_merge(so, other) for a non-empty `so` (the union's second step)
  void merge(const PySet& o) {
    if (&o == this || o.used == 0) return;
    if ((used + o.used) * 5 >= mask * 3) resize((used + o.used) * 2);
    if (used == 0) {  // empty target: same-size slot copy, else clean re-insert
      if (mask == o.mask) {
        table = o.table;
      } else {
        for (int64_t k : o.table)
          if (k != kEmpty) insert_clean(table, mask, k);
      }
      used = o.used;
      return;
    }
    for (int64_t k : o.table)
      if (k != kEmpty) add(k);
  }

  // The table `set(self)` (make_new_set -> set_merge into an empty set) would get:
  // same size -> identical slots; otherwise the keys re-inserted in slot order.
  void copy_in_place() {
    if (used == 0) { clear(); return; }
    size_t newsize = kMinSize;
    if (used * 5 >= (kMinSize - 1) * 3)
      while (newsize <= used * 2) newsize <<= 1;
    if (newsize == mask + 1) return;
    std::vector<int64_t> fresh(newsize, kEmpty);
    for (int64_t k : table)
      if (k != kEmpty) insert_clean(fresh, newsize - 1, k);
    table.swap(fresh);
    mask = newsize - 1;
  }

  template <class F>
  void for_each(F&& f) const {
    for (int64_t k : table)
      if (k != kEmpty) f(k);
  }
};

// ---------------------------------------------------------------- random.sample / choices
// random.sample(population, k) with n = len(population) > k (data_utils.py:92)
void py_sample(Mt& rng, const int64_t* pop, int64_t n, int64_t k, std::vector<int64_t>& out,
               std::vector<int64_t>& pool, std::vector<int64_t>& selected) {
  int64_t setsize = 21;
  if (k > 5) setsize += static_cast<int64_t>(pow(4.0, ceil(log(static_cast<double>(k * 3)) /
                                                            log(4.0))));
  if (n <= setsize) {
    pool.assign(pop, pop + n);
    for (int64_t i = 0; i < k; ++i) {
      const int64_t j = rng.randbelow(n - i);
      out.push_back(pool[j]);
      pool[j] = pool[n - i - 1];
    }
  } else {
    selected.clear();
    for (int64_t i = 0; i < k; ++i) {
      int64_t j = rng.randbelow(n);
      while (std::find(selected.begin(), selected.end(), j) != selected.end())
        j = rng.randbelow(n);
      selected.push_back(j);
      out.push_back(pop[j]);
    }
  }
}

// random.choices(population, k=k) (data_utils.py:94); n == 0 raises after one random()
bool py_choices(Mt& rng, const int64_t* pop, int64_t n, int64_t k, std::vector<int64_t>& out) {
  const double nf = static_cast<double>(n);
  for (int64_t i = 0; i < k; ++i) {
    const int64_t j = static_cast<int64_t>(floor(rng.random() * nf));
    if (j >= n) return false;  // IndexError: Cannot choose from an empty sequence
    out.push_back(pop[j]);
  }
  return true;
}

struct LayerResult {
  int64_t layers = 0, pad_len = 0, width = 0;
  std::vector<int64_t> neigh;   // [layers, pad_len, width], output order (deepest first)
  std::vector<int64_t> center;  // [layers, pad_len]
};

// node -> position map (the dict layer_nodes_map[i] of the reference; last write wins)
struct NodeIndex {
  std::unordered_map<int64_t, int64_t> idx;
  explicit NodeIndex(size_t n) { idx.reserve(n); }
  void set(int64_t node, int64_t i) { idx[node] = i; }
  int64_t get(int64_t node) const {
    auto it = idx.find(node);
    return it == idx.end() ? -1 : it->second;
  }
};

}  // namespace
}  // namespace gnn

using namespace gnn;

extern "C" int gnn_pyset_order(const int64_t* keys, int64_t n, int64_t* out, int64_t* n_out) {
  if ((n > 0 && (keys == nullptr || out == nullptr)) || n < 0 || n_out == nullptr) return GNN_E_ARG;
  try {
    PySet s;
    for (int64_t i = 0; i < n; ++i) {
      if (keys[i] < 0 || keys[i] >= (int64_t{1} << 61) - 1) return GNN_E_UNSUPPORTED;
      s.add(keys[i]);
    }
    int64_t m = 0;
    s.for_each([&](int64_t k) { out[m++] = k; });
    *n_out = m;
  } catch (const std::bad_alloc&) {
    return GNN_E_NOMEM;
  }
  return GNN_OK;
}

extern "C" int gnn_pyset_union_order(const int64_t* a, int64_t na, const int64_t* b, int64_t nb,
                                     int64_t* out, int64_t* n_out) {
  if (na < 0 || nb < 0 || n_out == nullptr || (na + nb > 0 && out == nullptr)) return GNN_E_ARG;
  try {
    PySet sa, sb;
    for (int64_t i = 0; i < na; ++i) {
      if (a[i] < 0) return GNN_E_UNSUPPORTED;
      sa.add(a[i]);
    }
    for (int64_t i = 0; i < nb; ++i) {
      if (b[i] < 0) return GNN_E_UNSUPPORTED;
      sb.add(b[i]);
    }
    sa.copy_in_place();
    sa.merge(sb);
    int64_t m = 0;
    sa.for_each([&](int64_t k) { out[m++] = k; });
    *n_out = m;
  } catch (const std::bad_alloc&) {
    return GNN_E_NOMEM;
  }
  return GNN_OK;
}

extern "C" int gnn_pyadj_build(const int64_t* src, const int64_t* dst, int64_t n_pairs,
                               int64_t n_nodes, int64_t* rowptr, int64_t* nbr) {
  if (n_pairs < 0 || n_nodes < 0 || rowptr == nullptr ||
      (n_pairs > 0 && (src == nullptr || dst == nullptr || nbr == nullptr)))
    return GNN_E_ARG;
  try {
    // per-node insertion streams in reference order: pair t adds dst to src's set, then
    // src to dst's set (data_utils.py:36-37) -- a stable counting sort of 2 n_pairs events
    std::vector<int64_t> start(static_cast<size_t>(n_nodes) + 1, 0);
    for (int64_t t = 0; t < n_pairs; ++t) {
      if (src[t] < 0 || src[t] >= n_nodes || dst[t] < 0 || dst[t] >= n_nodes) return GNN_E_ARG;
      ++start[src[t] + 1];
      ++start[dst[t] + 1];
    }
    for (int64_t v = 0; v < n_nodes; ++v) start[v + 1] += start[v];
    std::vector<int64_t> ev(static_cast<size_t>(2 * n_pairs));
    {
      std::vector<int64_t> pos(start.begin(), start.end() - 1);
      for (int64_t t = 0; t < n_pairs; ++t) {
        ev[pos[src[t]]++] = dst[t];
        ev[pos[dst[t]]++] = src[t];
      }
    }
    rowptr[0] = 0;
    std::vector<int64_t> deg(static_cast<size_t>(n_nodes), 0);
    // every node's set is independent: emulate them on a few host threads
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
      PySet s;
      for (;;) {
        const int64_t v0 = next.fetch_add(4096);
        if (v0 >= n_nodes) return;
        for (int64_t v = v0; v < std::min(n_nodes, v0 + 4096); ++v) {
          s.clear();
          for (int64_t e = start[v]; e < start[v + 1]; ++e) s.add(ev[e]);
          int64_t m = 0;
          s.for_each([&](int64_t k) { ev[start[v] + m++] = k; });  // iteration order, in place
          deg[v] = m;
        }
      }
    };
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < nt && n_nodes > 4096 * static_cast<int64_t>(t); ++t)
      pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
    int64_t o = 0;
    for (int64_t v = 0; v < n_nodes; ++v) {
      for (int64_t e = 0; e < deg[v]; ++e) nbr[o + e] = ev[start[v] + e];
      o += deg[v];
      rowptr[v + 1] = o;
    }
  } catch (const std::bad_alloc&) {
    return GNN_E_NOMEM;
  }
  return GNN_OK;
}

extern "C" int gnn_py_layer_sample(const int64_t* rowptr, const int64_t* nbr, int64_t n_nodes,
                                   const int64_t* nodes, int64_t n_batch, int32_t num_layers,
                                   int64_t num_neighs, int32_t is_gcn, uint32_t* mt_state,
                                   void** result) {
  if (result == nullptr) return GNN_E_ARG;
  *result = nullptr;
  if (rowptr == nullptr || mt_state == nullptr || n_nodes < 0 || n_batch < 0 || num_layers < 1 ||
      num_neighs < 0 || (n_batch > 0 && nodes == nullptr) || mt_state[624] > 624)
    return GNN_E_ARG;
  try {
    Mt rng;
    memcpy(rng.mt, mt_state, sizeof(rng.mt));
    rng.index = static_cast<int>(mt_state[624]);
    const int64_t width = num_neighs + (is_gcn ? 1 : 0);
    const int L = num_layers;
    std::vector<std::vector<int64_t>> centers(L + 1);  // layer_center_nodes
    std::vector<std::vector<int64_t>> samples(L);      // layer_neigh_nodes[i], flattened
    std::vector<NodeIndex> index_of;                   // layer_nodes_map[i]
    index_of.reserve(L);
    centers[0].assign(nodes, nodes + n_batch);
    std::vector<int64_t> cur(nodes, nodes + n_batch), draw, pool, selected;
    PySet layer_nodes, tmp;
    int status = GNN_OK;
    for (int i = 0; i < L; ++i) {
      index_of.emplace_back(cur.size());
      NodeIndex& map = index_of.back();
      samples[i].reserve(cur.size() * static_cast<size_t>(width));
      for (size_t idx = 0; idx < cur.size(); ++idx) {
        const int64_t node = cur[idx];
        if (node < 0 || node >= n_nodes) {
          status = GNN_E_ARG;  // the reference's defaultdict would yield an empty set
          break;
        }
        map.set(node, static_cast<int64_t>(idx));
        const int64_t* nb = nbr + rowptr[node];
        const int64_t deg = rowptr[node + 1] - rowptr[node];
        draw.clear();
        if (deg > num_neighs) {
          py_sample(rng, nb, deg, num_neighs, draw, pool, selected);
        } else if (!py_choices(rng, nb, deg, num_neighs, draw)) {
          status = GNN_E_EMPTY;
          break;
        }
        if (is_gcn) draw.push_back(node);
        else layer_nodes.add(node);
        samples[i].insert(samples[i].end(), draw.begin(), draw.end());
        // layer_nodes = layer_nodes.union(set(sample_neighs))
        tmp.clear();
        for (int64_t v : draw) tmp.add(v);
        layer_nodes.copy_in_place();
        layer_nodes.merge(tmp);
      }
      if (status != GNN_OK) break;
      cur.clear();
      layer_nodes.for_each([&](int64_t k) { cur.push_back(k); });
      centers[i + 1] = cur;
      layer_nodes.clear();
    }
    if (status == GNN_OK && n_batch == 0 && L > 1) status = GNN_E_ARG;  // len(X[0]) on []
    if (status != GNN_OK) {  // the generator still advanced, as the reference's would
      memcpy(mt_state, rng.mt, sizeof(rng.mt));
      mt_state[624] = static_cast<uint32_t>(rng.index);
      return status;
    }
    auto* res = new LayerResult();
    res->layers = L;
    res->width = width;
    res->pad_len = static_cast<int64_t>(centers[L - 1].size());  // len(layer_neigh_nodes[L-1])
    for (int i = 0; i < L - 1; ++i) {  // adj_nodes_pad cannot shorten a longer layer
      if (static_cast<int64_t>(centers[i].size()) > res->pad_len) {
        delete res;
        memcpy(mt_state, rng.mt, sizeof(rng.mt));
        mt_state[624] = static_cast<uint32_t>(rng.index);
        return GNN_E_RAGGED;
      }
    }
    const int64_t P = res->pad_len;
    res->neigh.assign(static_cast<size_t>(L * P * width), -1);
    res->center.assign(static_cast<size_t>(L * P), -1);
    for (int o = 0; o < L; ++o) {  // output slot o holds layer i = L-1-o
      const int i = L - 1 - o;
      int64_t* nm = res->neigh.data() + static_cast<size_t>(o) * P * width;
      int64_t* cm = res->center.data() + static_cast<size_t>(o) * P;
      if (i == L - 1) {  // global ids
        std::copy(samples[i].begin(), samples[i].end(), nm);
        std::copy(centers[i].begin(), centers[i].end(), cm);
      } else {  // positions in layer i+1's enumeration
        const NodeIndex& map = index_of[i + 1];
        for (size_t e = 0; e < samples[i].size(); ++e) nm[e] = map.get(samples[i][e]);
        for (size_t r = 0; r < centers[i].size(); ++r) cm[r] = map.get(centers[i][r]);
      }
    }
    memcpy(mt_state, rng.mt, sizeof(rng.mt));
    mt_state[624] = static_cast<uint32_t>(rng.index);
    *result = res;
  } catch (const std::bad_alloc&) {
    return GNN_E_NOMEM;
  }
  return GNN_OK;
}

extern "C" int gnn_py_layer_result_shape(const void* result, int64_t* dims) {
  if (result == nullptr || dims == nullptr) return GNN_E_ARG;
  const auto* r = static_cast<const LayerResult*>(result);
  dims[0] = r->layers;
  dims[1] = r->pad_len;
  dims[2] = r->width;
  return GNN_OK;
}

extern "C" int gnn_py_layer_result_copy(const void* result, int64_t* neigh_map,
                                        int64_t* center_map) {
  if (result == nullptr || neigh_map == nullptr || center_map == nullptr) return GNN_E_ARG;
  const auto* r = static_cast<const LayerResult*>(result);
  std::copy(r->neigh.begin(), r->neigh.end(), neigh_map);
  std::copy(r->center.begin(), r->center.end(), center_map);
  return GNN_OK;
}

extern "C" void gnn_py_layer_result_free(void* result) {
  delete static_cast<LayerResult*>(result);
}
