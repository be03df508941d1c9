// srt_comm.cpp -- RCCL communicator for the row-sharded multi-GPU build.
#include <cstring>

#include "srt_internal.h"

extern "C" {

srt_status srt_comm_unique_id(uint8_t out[128], srt_err *err) {
    (void)out;
    if (err) {
        std::memset(err, 0, sizeof *err);
        err->code = SRT_ERR_UNSUPPORTED;
        std::snprintf(err->msg, sizeof err->msg, "multi-GPU build not available in this build");
    }
    return SRT_ERR_UNSUPPORTED;
}

srt_status srt_comm_init(const uint8_t id[128], int nranks, int rank, int device, srt_comm **comm,
                         srt_err *err) {
    (void)id; (void)nranks; (void)rank; (void)device; (void)comm;
    return srt_comm_unique_id(nullptr, err);
}

void srt_comm_destroy(srt_comm *comm) { (void)comm; }

srt_status srt_plan_bind_comm(srt_plan *plan, srt_comm *comm, srt_err *err) {
    (void)plan; (void)comm;
    return srt_comm_unique_id(nullptr, err);
}

}  // extern "C"
