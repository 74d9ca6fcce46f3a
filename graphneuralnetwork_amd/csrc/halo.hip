// halo.hip -- the edge-cut halo exchange as a C-ABI entry (SURVEY 8(b) gnn_halo_alltoallv).
//
// One all-to-all-v of feature rows between the ranks of an edge-cut aggregation: rank p
// sends send_rows[q] rows to every rank q (contiguous blocks in peer order) and receives
// recv_rows[q] rows from each, with RCCL's ncclAllToAllv over xGMI (all peer links at once).
// This is what distributed.EdgeCutSpmm / EdgeCutGat run through torch.distributed's
// all_to_all_single on the nccl (= RCCL) backend; the entry lets a C caller of the library
// run the same exchange on its own communicator.
//
// The library does not link RCCL: the communicator belongs to whichever RCCL the caller
// loaded (PyTorch ships its own librccl.so), so ncclAllToAllv is resolved at the first call
// from the process -- the global scope, then an already-loaded librccl.so / librccl.so.1 --
// so that the call and the communicator come from the same library. An RCCL that is not
// loaded yet is never loaded here: it could not own the caller's communicator, so the entry
// returns GNN_E_COMM instead.
#include <dlfcn.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace gnn {

// ncclResult_t ncclAllToAllv(sendbuff, sendcounts[], sdispls[], recvbuff, recvcounts[],
//                            rdispls[], ncclDataType_t, ncclComm_t, hipStream_t)
typedef int (*AllToAllvFn)(const void*, const size_t*, const size_t*, void*, const size_t*,
                           const size_t*, int, void*, hipStream_t);
constexpr int kNcclFloat32 = 7;  // ncclFloat32 in rccl.h

static AllToAllvFn g_a2av = nullptr;
static std::once_flag g_a2av_once;

static void resolve_a2av() {
  void* f = dlsym(RTLD_DEFAULT, "ncclAllToAllv");
  const char* names[] = {"librccl.so", "librccl.so.1"};
  for (const char* nm : names) {
    if (f) break;
    void* h = dlopen(nm, RTLD_LAZY | RTLD_NOLOAD);
    if (h) f = dlsym(h, "ncclAllToAllv");
  }
  g_a2av = reinterpret_cast<AllToAllvFn>(f);
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_halo_rccl_path(char* buf, int64_t len) {
  std::call_once(g_a2av_once, resolve_a2av);
  if (!g_a2av) return GNN_E_COMM;
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(g_a2av), &info) || !info.dli_fname) return GNN_E_COMM;
  if (buf && len > 0) {
    int64_t i = 0;
    for (; i + 1 < len && info.dli_fname[i]; ++i) buf[i] = info.dli_fname[i];
    buf[i] = 0;
  }
  return GNN_OK;
}

extern "C" int gnn_halo_alltoallv_f32(const float* send, const int64_t* send_rows, float* recv,
                                      const int64_t* recv_rows, int64_t row_floats, int64_t world,
                                      void* comm, void* stream) {
  if (world < 1 || row_floats < 0 || !send_rows || !recv_rows || !comm) return GNN_E_ARG;
  std::vector<size_t> sc(world), sd(world), rc(world), rd(world);
  // element counts and running offsets must stay below 2^62 (no signed / size_t wrap)
  constexpr int64_t kMax = INT64_C(1) << 62;
  int64_t so = 0, ro = 0;
  for (int64_t q = 0; q < world; ++q) {
    if (send_rows[q] < 0 || recv_rows[q] < 0) return GNN_E_ARG;
    if (row_floats > 0 && (send_rows[q] > kMax / row_floats || recv_rows[q] > kMax / row_floats))
      return GNN_E_UNSUPPORTED;
    const int64_t s = send_rows[q] * row_floats, r = recv_rows[q] * row_floats;
    if (s > kMax - so || r > kMax - ro) return GNN_E_UNSUPPORTED;
    sc[q] = static_cast<size_t>(s);
    rc[q] = static_cast<size_t>(r);
    sd[q] = static_cast<size_t>(so);
    rd[q] = static_cast<size_t>(ro);
    so += s;
    ro += r;
  }
  if ((so && !send) || (ro && !recv)) return GNN_E_ARG;
  std::call_once(g_a2av_once, resolve_a2av);
  if (!g_a2av) return GNN_E_COMM;
  const int r = g_a2av(send, sc.data(), sd.data(), recv, rc.data(), rd.data(), kNcclFloat32, comm,
                       static_cast<hipStream_t>(stream));
  return r == 0 ? GNN_OK : GNN_E_COMM;
}
