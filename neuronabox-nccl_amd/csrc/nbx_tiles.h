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
// waiting for the slowest CU's fixed share (+4 % on config B in-process,
// profiles/r2/sweep_fold_r2_dyn_r2t.txt). A launch fetches exactly nTiles
// times (one per tile it runs), which is what the host adds to dynBase.
template <class Body>
__device__ __forceinline__ void forEachTile(const KArgs& a, uint64_t nTiles, Body body) {
  __shared__ uint32_t nxt[2];
  const bool dyn = a.dynCtr != nullptr;   // uniform
  uint64_t t = blockIdx.x;
  int par = 0;
  while (t < nTiles) {   // one copy of the body for both schedules
    if (dyn && threadIdx.x == 0) nxt[par] = atomicAdd(a.dynCtr, 1u) - a.dynBase + gridDim.x;
    body(t);
    if (dyn) {
      __syncthreads();
      t = nxt[par];
      par ^= 1;
    } else {
      t += gridDim.x;
    }
  }
}

}  // namespace nbx
