// sample.hip -- GraphSAGE neighbour sampling on gfx950 (the "next" row of SURVEY 8f): one
// frontier, one fanout (gnn_sample_neighbors). The draw itself is sample_kernels.hpp; the fused
// multi-hop batch (frontier + maps on the device, no host round trip between hops) is
// gnn_sample_layers in frontier.hip.
#include "sample_kernels.hpp"

using namespace gnn;

extern "C" int gnn_sample_neighbors(const int64_t* rowptr, const int32_t* col, int64_t n_graph,
                                    const int64_t* nodes, int64_t n, int64_t k, uint64_t seed,
                                    int64_t* out, int32_t* err_flag, void* stream) {
  if (n < 0 || k < 0 || n_graph < 0 || k > kMaxFanout) return GNN_E_ARG;
  if (n == 0 || k == 0) return GNN_OK;
  if (!rowptr || !col || !nodes || !out || !err_flag) return GNN_E_ARG;
  if ((n + 255) / 256 > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  launch_sample(rowptr, col, n_graph, nodes, n, nullptr, static_cast<int>(k), k, false, seed, out,
                err_flag, static_cast<hipStream_t>(stream));
  return launch_status();
}
