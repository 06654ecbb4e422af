// Data-parallel gradient exchange over RCCL (xGMI inside one node).
//
// The reference is single-process/single-device (I/train.py:58); this is new in the build
// (SURVEY.md §5, §8(e)).  One SUM all-reduce per step over the flat buffer
// [student grads (197,892) | DACP tau', score sums, counts | losses]  (~0.79 MB): small and
// latency-bound on xGMI, so it is issued as a single call on the step's stream (graph-
// capturable), right after the local backward and before the clip/Adam/EMA kernel which
// averages it (dad_step_apply with dp_world > 1).
#include <rccl/rccl.h>
#include <string.h>

#include "dad_common.h"

extern "C" {

int dad_comm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int dad_comm_get_unique_id(void* id_out) {
  if (!id_out) return DAD_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return DAD_E_COMM;
  memcpy(id_out, &id, sizeof(id));
  return DAD_OK;
}

int dad_comm_init(void** comm, int nranks, const void* id, int rank) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return DAD_E_ARG;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c;
  if (ncclCommInitRank(&c, nranks, uid, rank) != ncclSuccess) return DAD_E_COMM;
  *comm = (void*)c;
  return DAD_OK;
}

int dad_comm_allreduce_grad(void* comm, const dad_state* st, void* stream) {
  if (!comm || !st || !st->grad) return DAD_E_ARG;
  if (ncclAllReduce(st->grad, st->grad, DAD_GRAD_FLOATS, ncclFloat32, ncclSum, (ncclComm_t)comm,
                    (hipStream_t)stream) != ncclSuccess)
    return DAD_E_COMM;
  return DAD_OK;
}

int dad_comm_count(void* comm, int* nranks) {
  if (!comm || !nranks) return DAD_E_ARG;
  return ncclCommCount((ncclComm_t)comm, nranks) == ncclSuccess ? DAD_OK : DAD_E_COMM;
}

int dad_comm_allreduce_f32(void* comm, float* buf, size_t n, void* stream) {
  if (!comm || (!buf && n)) return DAD_E_ARG;
  if (ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, (ncclComm_t)comm, (hipStream_t)stream) != ncclSuccess)
    return DAD_E_COMM;
  return DAD_OK;
}

int dad_comm_destroy(void* comm) {
  if (!comm) return DAD_E_ARG;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? DAD_OK : DAD_E_COMM;
}

}  // extern "C"
