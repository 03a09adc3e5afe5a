// fm3d_internal.h -- entry points shared by the library's own translation units (not the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "fm3d.h"

// stage one frame pair (queryOffset 0) and queue the whole path with the survivor records compacted
// into recordsDev (device, capacity nA); returns without waiting (the context is then pending).  As
// fm3d_pipeline_submit for linked contexts: a member queues its front half only
int fm3d_internal_submit_to(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                            const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1,
                            const uint8_t* img2, int width, int height, fm3d_record* recordsDev);
// a link member's submitted pair whose leader has not launched it: its LM alone + records, queued
int fm3d_internal_flush(fm3d_ctx* c);
bool fm3d_internal_front_only(const fm3d_ctx* c);
// queue the whole path on the inputs fm3d_pipeline_upload staged
int fm3d_internal_enqueue(fm3d_ctx* c, fm3d_record* recordsDev);
// wait for the pending run: counts, guards, stats
int fm3d_internal_finish(fm3d_ctx* c, int* nKept, fm3d_pipeline_stats* stats);
// the survivor count of the queued run on the device (valid in stream order after the run)
const int* fm3d_internal_kept_dev(fm3d_ctx* c);
hipStream_t fm3d_internal_stream(fm3d_ctx* c);
int fm3d_internal_device(fm3d_ctx* c);
int fm3d_internal_prepare(fm3d_ctx* c);
// the device memory one context of this settings may grow to for a frame pair of nA x nB rows:
// its LM slabs (the largest launch) + a conservative estimate of the per-pair buffers
int fm3d_internal_memory_need(fm3d_ctx* c, int64_t nA, int64_t nB, int dim, int type, int width, int height,
                              size_t* bytes);
