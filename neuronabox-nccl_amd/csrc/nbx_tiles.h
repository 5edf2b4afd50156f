// nbx_tiles.h — tile scheduling shared by the reduce kernels and the stream
// ceiling kernels (device code; the host side is nbx::DynLaunch,
// nbx_internal.h / nbx_reduce.cc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nbx_kargs.h"

namespace nbx {

// Tile scheduling. Static: grid stride. Dynamic (a.dynCtr set by the host):
// workgroup b starts on tile b; every further tile comes from the stream's
// counter, fetched by thread 0 one tile ahead (into a double-buffered LDS
// word, so the atomic's latency hides behind the tile's loads) — CUs that
// stream faster take more tiles, and the grid finishes together instead of
// waiting for the slowest CU's fixed share (+4.8 % on config B in-process, +2-6 % in the library bench,
// profiles/r2/sweep_fold_r2_dyn_r2v.txt, profiles/r2/bench_dyn_ab_r2u.jsonl). A launch fetches exactly nTiles
// times (one per tile it runs), which is what the host adds to dynBase.
template <class Body>
__device__ __forceinline__ void forEachTile(const KArgs& a, uint64_t nTiles, Body body) {
  __shared__ uint32_t nxt[2];
  const bool dyn = a.dynCtr != nullptr;   // uniform
  uint64_t t = blockIdx.x;
  int par = 0;
  while (t < nTiles) {   // one copy of the body for both schedules
    // the next tile's index is requested before this tile's loads and only
    // consumed after its stores, so the atomic's round trip overlaps the tile
    // (writing it to LDS first made wave 0 wait for it before its loads)
    uint32_t got = 0;
    if (dyn && threadIdx.x == 0) got = atomicAdd(a.dynCtr, 1u);
    body(t);
    if (dyn) {
      if (threadIdx.x == 0) nxt[par] = got - a.dynBase + gridDim.x;
      __syncthreads();
      t = nxt[par];
      par ^= 1;
    } else {
      t += gridDim.x;
    }
  }
}

}  // namespace nbx
