// mmba_comm.cpp -- multi-GPU (one process per GPU) communicator.
//
// Round 1: the entry points exist so the ABI is complete; frame-sharded
// normal-equation reduction over RCCL is not wired yet and reports
// MMBA_ERR_UNSUPPORTED ("Multi-GPU").
#include <cstring>

#include "mmba_plan.h"

extern "C" {

int mmba_comm_unique_id(unsigned char out_id[128]) {
    if (!out_id) return MMBA_ERR_INVALID;
    std::memset(out_id, 0, 128);
    mmba::set_error("unsupported: RCCL sharding not wired in this build");
    return MMBA_ERR_UNSUPPORTED;
}

int mmba_plan_set_comm(mmba_plan *plan, int rank, int nranks, const unsigned char unique_id[128]) {
    (void)unique_id;
    if (!plan || rank < 0 || nranks <= 0 || rank >= nranks) return MMBA_ERR_INVALID;
    if (nranks == 1) return MMBA_OK;
    mmba::set_error("unsupported: RCCL sharding not wired in this build");
    return MMBA_ERR_UNSUPPORTED;
}

}  // extern "C"
