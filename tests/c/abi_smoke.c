/* abi_smoke.c — a plain C caller linked against libnbxccl.so exactly as an
 * NCCL user would be (include "nccl.h", -lnbxccl). Exercises only host-side
 * entry points so it runs without a GPU; prints "OK" on success. */
#include <stdio.h>
#include <string.h>

#include "nbx_reduce.h"
#include "nccl.h"

#define EXPECT(c)                                               \
  do {                                                          \
    if (!(c)) {                                                 \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                 \
    }                                                           \
  } while (0)

int main(void) {
  int v = 0;
  EXPECT(ncclGetVersion(&v) == ncclSuccess && v == NCCL_VERSION_CODE);
  EXPECT(pncclGetVersion(&v) == ncclSuccess && v == 21904);
  EXPECT(strcmp(ncclGetErrorString(ncclInvalidArgument),
                "invalid argument (run with NCCL_DEBUG=WARN for details)") == 0);
  ncclUniqueId id;
  EXPECT(ncclGetUniqueId(&id) == ncclSuccess);
  ncclComm_t comm = NULL;
  EXPECT(ncclCommInitRank(&comm, 4, id, 7) == ncclInvalidArgument);
  EXPECT(ncclAllReduce(NULL, NULL, 0, ncclFloat, ncclSum, NULL, NULL) == ncclInvalidArgument);
  EXPECT(ncclGroupStart() == ncclSuccess && ncclGroupEnd() == ncclSuccess);
  nbxDevRedOpFull op;
  EXPECT(nbxHostToDevRedOp(&op, ncclMax, ncclInt8, 1) == ncclSuccess);
  EXPECT(op.op == nbxDevMinMax && op.scalarArg == 0x7f);
  EXPECT(nbxHostToDevRedOp(&op, ncclAvg, ncclFloat32, 4) == ncclSuccess);
  EXPECT(op.op == nbxDevPreMulSum && op.scalarArg == 0x3e800000u);
  void* d[1] = {(void*)0x1000};
  const void* s[1] = {(void*)0x1000};
  EXPECT(nbxReduceMulti(d, 1, s, 1, 0, ncclFloat32, op, 1, 1, NULL) == ncclSuccess);  /* count 0 */
  EXPECT(nbxReduceMulti(d, 1, s, 0, 16, ncclFloat32, op, 1, 1, NULL) == ncclInvalidArgument);
  EXPECT(sizeof(ncclConfig_t) == 48 || sizeof(ncclConfig_t) == 56);
  printf("OK\n");
  return 0;
}
