// Internal helpers shared by the C-ABI translation units.
#pragma once

// Records `msg` as rt_last_error() for this thread and returns `code`.
int rt_internal_set_error(int code, const char* msg);

#include <cstdint>

struct rt_scene;
struct rt_camera;
struct rt_stats;
struct rt_group;

// Multi-GPU device groups (rt_multi.cpp; rt_set_devices in rt.h).
// A copy of the built scene `src` (host scene + trees) uploaded to `device`.
int rt_internal_replicate(const rt_scene* src, int device, rt_scene** out);
// Replicas on devices 1..n-1 of `primary` (device 0), one HIP stream per
// device and one RCCL communicator over the n devices.
int rt_internal_group_create(rt_scene* primary, int n, rt_group** out);
void rt_internal_group_destroy(rt_group* g);
int rt_internal_group_size(const rt_group* g);
// One frame on the group: row stripes on every device, one ncclGather of the
// slabs to device 0, un-interleave there, copy to out_rgb (W*H*3).  stats:
// work counters summed over the devices (nullable).
int rt_internal_group_render(rt_group* g, const rt_camera* cam, int aa, uint8_t* out_rgb, rt_stats* stats);
// n frames of one size in flight together on the group (each rank renders its stripes of all of them
// as one frame batch; one grouped RCCL call gathers them); outs[i]: W*H*3 host bytes.
int rt_internal_group_render_frames(rt_group* g, const rt_camera* cams, int n, int aa, uint8_t* const* outs,
                                    rt_stats* stats);
// RT_GROUP_VIRTUAL=1 (tests on a one-GPU box): a group of n ranks all on device 0, the gather done by
// device copies instead of RCCL -- everything of the group path except the RCCL call.
bool rt_internal_group_virtual();
int rt_internal_group_set_max_depth(rt_group* g, int depth);
