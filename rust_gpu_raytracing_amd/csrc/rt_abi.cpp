// rt_abi.cpp — host implementation of include/rt_abi.h.
//
// Replaces the wgpu side of the reference's per-frame path:
//   DataBuffers (src/buffers.rs:140-596)  -> hipMalloc'd device buffers, updated
//                                            through a pinned staging buffer with
//                                            hipMemcpyAsync on the context stream
//   Renderer::compute_frame (src/renderer.rs:201-252)
//                                         -> Params shadow + hipLaunchKernelGGL
// Stream order gives the same visibility guarantees as wgpu's queue order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_kernel_args.h"
#include "rt_scene_math.h"
#include "sphere_bvh.h"
#include "tri_cone.h"
#include "tri_qnode.h"

hipError_t rt_launch_math_selftest(uint32_t which, unsigned long long* mismatches, uint32_t* first_bad,
                                   hipStream_t stream);
hipError_t rt_launch_pathtrace(const KernelArgs& ka, int mode, bool tris, uint32_t threads, size_t lds_bytes,
                               uint32_t blocks, hipStream_t stream);
hipError_t rt_pathtrace_pick_config(int mode, bool tris, size_t lds_bytes, size_t lds_bytes_per_thread,
                                    uint32_t force_threads, uint32_t waves_cap, uint32_t* threads,
                                    int* blocks_per_cu);
hipError_t rt_launch_edit(const float* model, const uint32_t* tri_object, const uint32_t* sub_object,
                          const uint2* object_tris, const rt_scene::Placement* place, uint32_t object_count,
                          uint32_t n_tri, uint32_t n_sub, RtTriangleHot* tris, float4* bounds, RtSubObject* subs,
                          RtObject* objects, hipStream_t stream);
hipError_t rt_launch_quantize_tri_nodes(const SphereBvhNode* nodes, uint32_t n, const uint32_t* src,
                                        const uint32_t* skip, uint32_t n_out, SphereBvhNode* out32, uint4* q,
                                        float4* grid, hipStream_t stream);
hipError_t rt_launch_refit(SphereBvhNode* nodes, const SubObjectPrim* prims, const RtSubObject* subs,
                           const uint32_t* order, const uint32_t* level_offsets, uint32_t n_levels, float* extent_out,
                           hipStream_t stream);
hipError_t rt_launch_tri_leafcert(const SubObjectPrim* prims, uint32_t n_prims, const RtSubObject* subs,
                                  const RtTriangleHot* tris, uint32_t n_tri, TriLeafCert* out, hipStream_t stream);
hipError_t rt_launch_tri_leaftris(const SubObjectPrim* prims, uint32_t n_prims, const RtTriangleHot* tris,
                                  uint32_t n_tri, uint4* out, hipStream_t stream);
hipError_t rt_launch_primary(const KernelArgs& ka, int mode, bool tris, size_t lds_bytes, uint32_t threads,
                             uint32_t min_waves, hipStream_t stream);
hipError_t rt_launch_brute_wf(const KernelArgs& ka, bool tris, bool scalar_stream, size_t lds_bytes, uint32_t blocks,
                              hipStream_t stream);
size_t rt_brute_wf_tile_bytes(bool scalar_stream);
uint32_t rt_brute_wf_chunk();
hipError_t rt_launch_resolve(float4* accum, uint32_t* output, const float4* light, uint32_t width, uint32_t height,
                             uint32_t tiles_x, uint32_t owned_tiles, uint32_t rank, uint32_t world, uint32_t k0,
                             uint32_t samples, uint32_t frames, unsigned long long* clock, hipStream_t stream);
hipError_t rt_launch_pack_output(uint32_t* output, uint32_t* packed, uint32_t width, uint32_t height, uint32_t tiles_x,
                                 uint32_t n_tiles, uint32_t first_rank, uint32_t ranks, uint32_t world,
                                 uint64_t stride_px, uint32_t skip_rank, bool unpack, hipStream_t stream);
hipError_t rt_launch_pack(const float4* accum, float4* dst, uint32_t width, uint32_t height, uint32_t tiles_x,
                          uint32_t owned_tiles, uint32_t rank, uint32_t world, hipStream_t stream);
hipError_t rt_launch_unpack(const float4* src, float4* accum, uint32_t* output, uint32_t width, uint32_t height,
                            uint32_t tiles_x, uint32_t n_tiles, uint32_t first_rank, uint32_t ranks, uint32_t world,
                            uint64_t stride_px, uint32_t skip_rank, float divisor, hipStream_t stream);

static_assert(sizeof(rt_params) == 48, "Params is 48 bytes (src/buffers.rs:9-22)");
static_assert(sizeof(rt_ray_camera) == 16, "RayCamera is 16 bytes");
static_assert(sizeof(rt_ray) == 16, "Ray is 16 bytes");
static_assert(sizeof(rt_scene_sphere) == 32, "SceneSphere is 32 bytes");
static_assert(sizeof(rt_scene_triangle) == 112, "SceneTriangle is 112 bytes");
static_assert(sizeof(rt_scene_material) == 32, "SceneMaterial is 32 bytes");
static_assert(sizeof(rt_object_info) == 48, "ObjectInfo is 48 bytes");
static_assert(sizeof(rt_sub_object_info) == 32, "SubObjectInfo is 32 bytes");
static_assert(sizeof(rt_scene_material) == sizeof(RtMaterial), "material record");
static_assert(sizeof(rt_object_info) == sizeof(RtObject), "object record");
static_assert(sizeof(rt_sub_object_info) == sizeof(RtSubObject), "sub-object record");

namespace {

constexpr size_t kLdsSceneBudget = 64 * 1024;    // mode 1: spheres/materials/objects/sphere BVH per workgroup
constexpr size_t kLdsAccelBudget = 150 * 1024;   // mode 2: + triangle accelerator (one 1024-thread workgroup per CU)
// d_counter: [0] the ray counter, [1, 1 + kDiagCounters) the diagnostic
// counters of RT_DIAG / RT_DIAG_TAIL builds (KernelArgs::diag), then the
// per-wave (queue dry, end) records of RT_DIAG_TAIL builds: room for 65,536 waves.
constexpr size_t kDiagCounters = kDiagHeaderWords;
constexpr size_t kDiagWaveRecords = 2 * 65536;
constexpr size_t kCounterWords = 1 + kDiagCounters + kDiagWaveRecords;
// Tile queue: counters per stripe (pathtrace.hip, claim_tile), 256 B apart;
// kQueueStripes = 4 per XCD by default (measured: C2 0.599 ms at 8, 0.595 at 32; C1
// 0.076 -> 0.058 ms), up to kQueueStripesMax (RT_QUEUE_STRIPES).
constexpr uint32_t kQueueStripes = 32;
// Triangle-walk distance pruning: a node is skipped once its (inflated) box
// is entered beyond best * (1 + kTriPruneRho) + kTriPruneAbs * (|o| + extent) / |d|.
constexpr float kTriPruneRho = 1.0f / 64.0f;
constexpr uint32_t kQueueStripesMax = 64;
constexpr uint32_t kQueueStride = 64;
// A wave goes back to shading once at most this many of its 64 lanes are still
// traversing (pathtrace.hip, step 4 of the kernel loop). The longer a trace is
// against a shading pass, the earlier it pays to shade the finished lanes
// (measured: sphere scenes 8, C2 slower at 12+ until round 6's block group tests, since then 12:
// C2 0.2474 -> 0.2448 ms, 10 / 14 / 20: 0.2456 / 0.2444 / 0.2468, profiles/r06/r06v, r06w;
// triangle accelerator in LDS
// 24, C3/C4 -2%; in global memory 32, C5 -10%; with the pruned octant walk of round 3,
// 48: C5 5.95 -> 5.72 ms, profiles/r03_ah/knobs_c5b.jsonl; C3 unchanged at 24-32).
// certified: walks from global memory with the certified pruning, whose
// traces visit the box-culling node set (about twice the relative slack's): they return to
// shading later and batch their leaves earlier (C5 13.0 -> 11.1 ms per frame at 56 / 3, 10.7 at 56 / 4
// once the certificate test moved into the leaf batch;
// profiles/r04/r04_f/ab.jsonl; the slack keeps round 3's 48 / 5).
uint32_t trav_threshold_for(int lds_mode, bool tris, bool certified) {
    if (!tris) return 12;
    return lds_mode == 2 ? 24 : certified ? 56 : 48;
}
// Triangle scenes test deferred leaves once this many eighths of the
// traversing lanes hold one (pathtrace.hip, leaf_step): later for an LDS
// accelerator, earlier when the leaf's loads go to global memory anyway.
// Re-measured with 20-frame launches (profiles/archive/r02_s4/r02_s4k, r02_s4l):
// mode 2 at 6 (C4 -2.3% against 7, C3 within 0.3%), modes 0/1 at 5 (C5 -2.9%
// against 6; 4 and 3 within 0.4% of 5); certified walks at 4 (above; 3 before the certificate
// test moved into the leaf batch, profiles/r04/r04_k).
uint32_t leaf_batch_for(int lds_mode, bool certified) { return lds_mode == 2 ? 6 : certified ? 4 : 5; }
// Instances with the triangle accelerator in global memory: the same once the
// tile queue is empty, when the wave goes back to shading only if some lane
// has finished and after at least kDefaultDrainMinSteps traversal steps
// (threshold 0: traverse to the end, as the other instances do).
constexpr uint32_t kDefaultDrainThreshold = 32;
constexpr uint32_t kDefaultDrainMinSteps = 64;
// Tile claim order: 0 = tile index order, 1 = cost-ordered (most rays first,
// sorted on the device from the previous frame's per-tile ray counts).
constexpr uint32_t kDefaultTileSchedule = 1;
constexpr uint64_t kSchedMinTilesPerWave = 4;
// Frame batching (rt_set_frame_batch): at most this many frames per launch.
constexpr uint32_t kMaxFrameBatch = 64;
// Frame-parallel batches (every (frame, tile) its own queue unit, lights resolved
// in order afterwards) up to this many frames x samples; larger batches run each
// pixel's frames back to back on one lane.
constexpr uint32_t kMaxParallelLights = 64;

}  // namespace

// The last error of a call without a context (rt_create, the scene builders).
thread_local std::string g_create_error;
void rt_set_global_error(const std::string& msg) { g_create_error = msg; }

namespace {

constexpr uint32_t kClockSlots = 4096;
constexpr uint32_t kClockWords = 4;  // per timed launch: path kernel {~start, end}, resolve kernel {~start, end}

}  // namespace

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t width = 0, height = 0;
    uint64_t n_pixels = 0;
    uint32_t rank = 0, world = 1;
    uint32_t tiles_x = 0, tiles_y = 0, owned_tiles = 0;

    rt_params params{};  // shadow of binding 0
    uint32_t k = 1;      // Renderer::accumulation_index (src/renderer.rs:37)
    rt_ray_camera camera{};
    // frame batching (rt_set_frame_batch): queued rt_compute_frame calls
    uint32_t frame_batch = RT_DEFAULT_FRAME_BATCH;  // frames per launch at most (1: one launch per frame)
    uint32_t pending_frames = 0;  // queued, not yet launched (their k already advanced)
    uint32_t pending_bounces = 0;
    bool frame_parallel = true;     // tuning "frame_parallel" 0: batches run frames back to back per lane
    float4* d_frame_light[2] = {};    // frame-parallel batch lights (by batch parity), owned px x frames x samples
    size_t frame_light_cap = 0;       // float4 entries, each
    // overlapped batches (dispatch_frames): batch i runs on streams[i % 2]
    hipStream_t aux_stream = nullptr;
    hipEvent_t ev_resolved[2] = {};   // after batch i's resolve (i % 2)
    hipEvent_t ev_aux_done = nullptr; // after the last work issued on aux_stream
    hipEvent_t ev_primary = nullptr;  // a point of the primary stream an aux batch waits for
    bool aux_outstanding = false;     // aux work the primary stream has not been ordered after yet
    bool primary_dirty = true;        // primary-stream work since then that an aux batch must follow
    uint64_t batches = 0;             // frame-parallel batches launched
    bool batch_overlap = true;        // tuning "batch_overlap" 0: every batch on the primary stream
    bool stage_subs = true;           // tuning "stage_subs" 0: mode 2 leaves read sub-objects from global
    // device memory the batch buffers (frame lights, primary records) may take: a batch that
    // would need more is rendered as several launches (dispatch_batch); tuning "batch_memory_mb"
    size_t batch_budget = 0;
    // 16-B quantized triangle nodes for walks from global memory (tuning "tri_qnodes" 0: the 32-B nodes)
    bool use_qnodes = true;
    bool qnodes_dirty = true;          // the binary accelerator changed since the copy was made
    bool derived_octants = false, derived_qnodes = false;  // what the last derivation produced
    uint4* d_tri_qnodes = nullptr;
    float4* d_tri_qgrid = nullptr;
    size_t qnodes_cap = 0;
    bool batch_schedule = false;      // tuning "batch_schedule" 1: cost-ordered claims in batches too
    // a tile's frames claimed one after another (C3 -12%, C4 -8%, C5 -4%, C2 -1.8% per frame
    // against frame-major, profiles/archive/r02_knobs2); tuning "unit_tile_major" 0: frame-major
    bool unit_tile_major = true;

    uint32_t cap_mat = 0, cap_sph = 0, cap_tri = 0, cap_obj = 0, cap_sub = 0;
    // extents the kernel clamps against (>= 1 so clamps never underflow)
    uint32_t n_mat_dev = 1, n_tri_dev = 1, n_sub_dev = 1;

    float4* d_rays = nullptr;
    float4* d_accum = nullptr;
    uint32_t* d_out = nullptr;
    unsigned long long* d_counter = nullptr;
    uint32_t* d_queue = nullptr;  // [stream][2] x kQueueStripesMax tile-queue counters, kQueueStride apart
    uint32_t queue_parity[2] = {0, 0};  // per stream: which half its next launch uses (the launch zeroes the other)
    uint32_t queue_stripes = kQueueStripes;  // tuning "queue_stripes"
    int n_cu = 0;
    bool force_global_scene = false;   // tuning "scene_in_lds" 0
    size_t occ_lds_bytes = 0;
    int occ_mode = -1;
    bool occ_tris = false;
    size_t occ_stack_pt = 0;
    int max_lds_mode = 2;               // tuning "lds_mode": highest staging mode allowed
    int occ_blocks_per_cu = 0;
    uint32_t occ_threads = 0;
    uint32_t force_threads = 0;        // tuning "block_threads"; 0 = pick by occupancy
    uint32_t waves_cap = 0;            // tuning "waves_per_cu"; 0 = default cap
    uint32_t trav_threshold = 0;  // tuning "trav_threshold"; 0 = by scene (trav_threshold_for)
    uint32_t drain_threshold = kDefaultDrainThreshold;  // tuning "drain_threshold"
    uint32_t drain_min_steps = kDefaultDrainMinSteps;   // tuning "drain_min_steps"
    uint32_t leaf_batch = 0;  // tuning "leaf_batch", in eighths; 0 = by scene (leaf_batch_for)
    // cost-ordered tile schedule (rt_set_tile_schedule), double-buffered by
    // launch parity: launch L records costs[L&1], reads order[L&1], and its
    // first idle workgroup sorts costs[~L&1] (launch L-1's) into order[~L&1]
    uint32_t tile_schedule = kDefaultTileSchedule;  // rt_set_tile_schedule / tuning "tile_schedule"
    // per stream (launches on the auxiliary stream keep their own history):
    uint32_t* d_tile_sched[2] = {};    // costs[2][n], orders[2][n], flags[2] (n = owned tiles)
    uint64_t sched_launches[2] = {};   // launches since the schedule was (re)set
    uint32_t last_blocks = 0, last_lds = 0;
    uint32_t last_passes = 0;  // RT_PASS_* of the last dispatch
    float4* d_slot_sph = nullptr;        // kernel-ordered spheres (sphere_bvh.h)
    uint32_t* d_slot_orig = nullptr;
    uint32_t* d_sph_mat = nullptr;       // by original index
    SphereBvhNode* d_bvh = nullptr;
    std::vector<rt_scene_sphere> h_sph;  // host copy: the BVH is rebuilt from it
    bool slots_dirty = true;
    uint32_t slots_count = 0xffffffffu;  // sphere_count the slots were built for
    bool use_bvh = true;                 // tuning "sphere_bvh" 0: the brute-force sweep only
    bool sphere_octants = true;          // tuning "sphere_octants" 0: one BVH layout
    bool sphere_box_order = true;        // tuning "sphere_box_order" 0: octant layouts keep bmin/bmax
    bool sphere_boxes_ordered = false;   // the uploaded layouts store (near, far) corners
    bool slots_sphere_only = false;      // the uploaded slots were laid out for the sphere-only kernels
    uint32_t sphere_leaf_max = 0;        // tuning "sphere_leaf"; 0 = default
    uint32_t n_always = 0, n_nodes = 0, n_slots = 0;
    float sphere_extent = 0.0f;
    float sphere_rmin = 0.0f, sphere_rmax = 0.0f;
    // triangle accelerator over (object, sub-object) pairs (sphere_bvh.h)
    SphereBvhNode* d_tri_bvh = nullptr;
    SubObjectPrim* d_tri_prims = nullptr;
    size_t tri_bvh_cap = 0, tri_prims_cap = 0;
    bool tri_dirty = true;
    uint32_t tri_count_built = 0xffffffffu;
    bool use_tri_bvh = true;  // tuning "tri_bvh" 0: the reference's sweep
    // Direction-ordered layouts of the binary accelerator for walks from global memory (LDS
    // modes 0/1; order_bvh_by_octant): per position of the 8 layouts the base node and the
    // layout's skip link (host-built with the tree), and the 32-B copy derived from the base
    // nodes on the device after every upload or refit (with the quantized copy).
    // tuning "tri_octants" 0: one layout.
    bool use_tri_octants = true;
    uint32_t* d_tri_src8 = nullptr;
    uint32_t* d_tri_skip8 = nullptr;
    SphereBvhNode* d_tri_bvh8 = nullptr;
    size_t tri_src8_cap = 0, tri_skip8_cap = 0, tri_bvh8_cap = 0;
    bool tri_octants_built = false;  // d_tri_src8 / d_tri_skip8 describe the current tree
    // rt_set_triangle_pruning: distance pruning of the triangle walk: 1 =
    // certified by the leaf certificates (default, exact), 0 = box culling only, 2 = the round-3
    // relative slack (not exact: only this explicit call selects it)
    int tri_prune_mode = 1;
    // certified pruning (tri_cone.h): one certificate per leaf record, rebuilt on the device
    // after any change of the accelerator or the triangles
    TriLeafCert* d_tri_lcert = nullptr;
    size_t tri_lcert_cap = 0;
    bool cones_dirty = true;
    // cooperative leaf batches of the walks from global memory (pathtrace.hip coop_leaf_batch):
    // the leaves' triangle blocks, rebuilt with the certificates; tuning "coop_leaves" 0:
    // per-lane leaf tests
    bool use_coop_leaves = true;
    uint4* d_tri_ltris = nullptr;
    size_t tri_ltris_cap = 0;
    bool ltris_dirty = true;
    // rt_set_brute_force: the reference's own sweeps (BASELINE config 5): 0 off, 1 LDS-tiled, 2
    // through the scalar cache (rt_brute_wf_kernel<tris, stream>)
    int brute = 0;
    // coherent primary rays (rt_primary_kernel): tuning "primary_pass" 1 / 0 force on / off, -1 by scene
    int primary_pass = -1;
    // Workgroup size of the pre-pass where the accelerator is walked from global memory (modes
    // 0/1): its packet walks are chains of dependent node loads, so resident waves are what
    // count; at 1024 threads and ~69 VGPRs only one workgroup (16 waves) fits a CU, at 256 seven
    // (28 waves): C5 5.69 -> 5.24 ms per frame (profiles/r03_ai/ab_c5_pthreads.jsonl); held to
    // 64 VGPRs, eight waves per SIMD (32 per CU): 5.04 ms (profiles/r03_aj/ab_c5_pthreads.jsonl).
    // tunings "primary_threads" 64 / 128 / 256 / 512 / 1024 and "primary_waves" 0 / 8.
    uint32_t primary_threads = 256;
    uint32_t primary_min_waves = 8;
    // a tile's frames on consecutive pre-pass waves, whose packets walk nearly the same nodes:
    // C5 5.02 -> 4.93 ms (profiles/r03_al/ab_c5_ptm.jsonl); tuning "primary_tile_major" 0: frame-major
    bool primary_tile_major = true;
    uint4* d_primary[2] = {};   // per batch parity (overlapped batches), owned px x frames x samples records
    size_t primary_cap = 0;
    // sub-object bytes of the brute-force launches: [0] SURVEY §8d's tile-streaming convention,
    // [1] what the sweeps read from L2
    unsigned long long* d_stream = nullptr;
    // the brute-force wavefront (rt_brute_wf_kernel)
    float4* d_brute_paths = nullptr;
    uint32_t* d_brute_queue = nullptr;
    uint32_t* d_brute_counts = nullptr;
    size_t brute_paths_cap = 0, brute_queue_cap = 0, brute_counts_cap = 0;
    uint32_t tri_nodes = 0, tri_prim_count = 0;
    float* d_tri_extent = nullptr;   // margin extent, in device memory (refit updates it)
    uint32_t* d_tri_order = nullptr; // node indices by depth, deepest level first (refit)
    uint32_t* d_tri_level_off = nullptr;
    size_t tri_order_cap = 0, tri_level_cap = 0;
    uint32_t tri_levels = 0;
    // device-side edit path (scene_edit.hip): normalised points per triangle,
    // triangle/sub-object -> object maps, per-object triangle ranges, placements
    float* d_model = nullptr;
    uint32_t model_tris = 0;
    bool models_valid = false;  // rt_set_object_models since the last object / sub-object range change
    uint32_t* d_tri_object = nullptr;
    uint32_t* d_sub_object = nullptr;
    uint2* d_object_tris = nullptr;
    rt_scene::Placement* d_place = nullptr;
    float4* d_tri_bounds = nullptr;   // per-triangle min/max (SceneTriangle's host-only fields)
    bool geom_on_device = false;      // device edits are newer than h_obj / h_sub
    RtMaterial* d_mat = nullptr;
    RtObject* d_obj = nullptr;
    RtSubObject* d_sub = nullptr;
    RtTriangleHot* d_tri = nullptr;
    uint32_t* d_tex = nullptr;
    uint32_t tex_w = 0, tex_h = 0, tex_layers = 0;
    uint32_t* d_env = nullptr;
    uint32_t env_w = 0, env_h = 0;
    uint32_t env_uniform = 3;  // bit 0: every row one colour, bit 1: every column (sample_env skips u / v)
    float* d_srgb = nullptr;

    // host-side copies used for validation of index ranges
    std::vector<rt_object_info> h_obj;
    std::vector<rt_sub_object_info> h_sub;

    // pinned staging (one buffer, reused after its last copy completes)
    void* pinned = nullptr;
    size_t pinned_cap = 0;
    hipEvent_t staging_done = nullptr;
    bool staging_busy = false;

    // timing
    bool timing = false;
    bool gen_rays = false;  // rt_update_camera_matrices: primary rays computed on the device
    float inv_proj[16] = {}, inv_view[16] = {};
    // launch timing (rt_set_timing): each timed launch's kernel span on the device
    // clock -- the first workgroup's start to the last one's end (s_memrealtime) --
    // in a ring of slots read back in bulk; HIP events would time each launch from
    // the moment its stream reached it, which overlapped batches make meaningless
    unsigned long long* d_clock = nullptr;  // kClockSlots x {path: ~min start, max end; resolve: the same}
    std::vector<uint32_t> clock_pending;    // slots of timed launches not yet read back
    uint32_t clock_next = 0;
    double wall_khz = 100000.0;             // device wall clock rate (hipDeviceAttributeWallClockRate)
    double total_ms = 0.0;
    uint64_t n_timed = 0;
    double resolve_total_ms = 0.0;  // rt_resolve_frames_kernel spans of the timed batches
    uint64_t n_resolve_timed = 0;
    float last_ms = 0.0f;

    std::string err;
};

static int flush_frames(rt_ctx* ctx);

// Orders the primary stream after everything issued on the auxiliary stream
// (overlapped batches): every call other than rt_compute_frame runs this first.
static hipError_t join_aux(rt_ctx* ctx) {
    if (!ctx->aux_outstanding) return hipSuccess;
    ctx->aux_outstanding = false;
    return hipStreamWaitEvent(ctx->stream, ctx->ev_aux_done, 0);
}

namespace {

int fail(rt_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg; else g_create_error = msg;
    return code;
}

int hip_fail(rt_ctx* ctx, const char* what, hipError_t e) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(ctx, RT_E_HIP, m);
}

#define RT_HIP(ctx, call)                                \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return hip_fail(ctx, #call, e_); \
    } while (0)

void srgb_table(float out[256]) {
    // IEC 61966-2-1 decode of an 8-bit Rgba8UnormSrgb channel, rounded to f32.
    for (int i = 0; i < 256; i++) {
        const double c = (double)i / 255.0;
        const double l = c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4);
        out[i] = (float)l;
    }
}

uint32_t owned_tile_count(uint32_t n_tiles, uint32_t rank, uint32_t world) {
    if (rank >= n_tiles) return 0;
    return (n_tiles - rank + world - 1) / world;
}

// Returns a pinned host region of at least `bytes`, waiting for any copy
// still reading the previous contents.
int staging(rt_ctx* ctx, size_t bytes, void** out) {
    if (ctx->staging_busy) {
        RT_HIP(ctx, hipEventSynchronize(ctx->staging_done));
        ctx->staging_busy = false;
    }
    if (bytes > ctx->pinned_cap) {
        if (ctx->pinned) RT_HIP(ctx, hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_cap = 0;
        size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
        RT_HIP(ctx, hipHostMalloc(&ctx->pinned, cap, hipHostMallocDefault));
        ctx->pinned_cap = cap;
    }
    *out = ctx->pinned;
    return RT_OK;
}

int staged_copy(rt_ctx* ctx, void* dst, size_t bytes) {
    if (bytes == 0) return RT_OK;
    RT_HIP(ctx, hipMemcpyAsync(dst, ctx->pinned, bytes, hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(ctx, hipEventRecord(ctx->staging_done, ctx->stream));
    ctx->primary_dirty = true;  // an overlapped batch issued later must follow this copy
    ctx->staging_busy = true;
    return RT_OK;
}

int upload_raw(rt_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return RT_OK;
    void* p;
    int rc = staging(ctx, bytes, &p);
    if (rc) return rc;
    std::memcpy(p, src, bytes);
    return staged_copy(ctx, dst, bytes);
}

int upload_spheres(rt_ctx* ctx, const rt_scene_sphere* s, uint32_t n) {
    if (n == 0) return RT_OK;
    std::copy(s, s + n, ctx->h_sph.begin());
    ctx->slots_dirty = true;  // slots + BVH are rebuilt at the next dispatch
    return RT_OK;
}

// Rebuild the kernel's sphere slots (brute-force set + BVH) for the first
// `count` spheres and upload them, stream-ordered before the next launch.
int refresh_sphere_slots(rt_ctx* ctx, uint32_t count, bool sphere_only) {
    if (!ctx->slots_dirty && ctx->slots_count == count && ctx->slots_sphere_only == sphere_only) return RT_OK;
    SphereSlots sl;
    build_sphere_slots(ctx->h_sph.data(), count, ctx->use_bvh, &sl, ctx->sphere_leaf_max);
    std::vector<uint32_t> mat(count);
    for (uint32_t i = 0; i < count; i++) mat[i] = ctx->h_sph[i].material_index;
    std::vector<SphereBvhNode> oct;  // 8 direction-ordered copies; layout 0 alone is a complete walk too
    // boxes stored as (near, far) corners per octant when that is exact (rt_bvh_slab.h);
    // only the sphere-only kernels read them that way, so only for scenes without objects
    const bool box_order = ctx->sphere_box_order && sphere_only && box_layout_orderable(sl.nodes);
    order_bvh_by_octant(sl.nodes, &oct, box_order);
    int rc;
    if ((rc = upload_raw(ctx, ctx->d_slot_sph, sl.slot_sph.data(), sl.slot_sph.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_slot_orig, sl.slot_orig.data(), sl.slot_orig.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_sph_mat, mat.data(), mat.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_bvh, oct.data(), oct.size() * sizeof(SphereBvhNode))))
        return rc;
    ctx->n_always = sl.n_always;
    ctx->n_slots = (uint32_t)sl.slot_orig.size();
    ctx->n_nodes = (uint32_t)sl.nodes.size();
    ctx->sphere_boxes_ordered = box_order;
    ctx->sphere_extent = sl.extent;
    ctx->sphere_rmin = sl.r_min;
    ctx->sphere_rmax = sl.r_max;
    ctx->slots_dirty = false;
    ctx->slots_count = count;
    ctx->slots_sphere_only = sphere_only;
    return RT_OK;
}

// After device-side edits (rt_update_objects) the host copies of the object and
// sub-object records are stale; read them back before anything host-side uses
// their bounds.
int sync_host_geometry(rt_ctx* ctx) {
    if (!ctx->geom_on_device) return RT_OK;
    if (!ctx->h_obj.empty())
        RT_HIP(ctx, hipMemcpyAsync(ctx->h_obj.data(), ctx->d_obj, ctx->h_obj.size() * 48, hipMemcpyDeviceToHost,
                                   ctx->stream));
    if (!ctx->h_sub.empty())
        RT_HIP(ctx, hipMemcpyAsync(ctx->h_sub.data(), ctx->d_sub, ctx->h_sub.size() * 32, hipMemcpyDeviceToHost,
                                   ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->geom_on_device = false;
    return RT_OK;
}

// Rebuild the triangle accelerator for the first `object_count` objects when
// objects or sub-objects changed (the boxes it culls with are theirs).
int refresh_tri_accel(rt_ctx* ctx, uint32_t object_count) {
    if (!ctx->use_tri_bvh || object_count == 0) return RT_OK;
    if (!ctx->tri_dirty && ctx->tri_count_built == object_count) return RT_OK;
    int rc0 = sync_host_geometry(ctx);
    if (rc0) return rc0;
    auto ensure = [&](void** p, size_t* cap, size_t bytes) -> int {
        if (bytes <= *cap && *p) return RT_OK;
        RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (*p) RT_HIP(ctx, hipFree(*p));
        *p = nullptr;
        *cap = 0;
        const size_t alloc = bytes < 256 ? 256 : bytes;
        RT_HIP(ctx, hipMalloc(p, alloc));
        *cap = alloc;
        return RT_OK;
    };
    int rc;
    TriangleAccel acc;
    build_triangle_accel(ctx->h_obj.data(), object_count, ctx->h_sub.data(), (uint32_t)ctx->h_sub.size(), &acc);
    const size_t nb = acc.nodes.size() * sizeof(SphereBvhNode), pb = acc.prims.size() * sizeof(SubObjectPrim);
    if ((rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_bvh), &ctx->tri_bvh_cap, nb)) ||
        (rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_prims), &ctx->tri_prims_cap, pb)) ||
        (rc = upload_raw(ctx, ctx->d_tri_bvh, acc.nodes.data(), nb)) ||
        (rc = upload_raw(ctx, ctx->d_tri_prims, acc.prims.data(), pb)))
        return rc;
    ctx->qnodes_dirty = true;
    ctx->cones_dirty = true;
    ctx->ltris_dirty = true;
    ctx->tri_nodes = (uint32_t)acc.nodes.size();
    ctx->tri_prim_count = (uint32_t)acc.prims.size();
    ctx->tri_octants_built = false;
    if (ctx->use_tri_octants && acc.nodes.size() > 1 && acc.nodes.size() * 8 < (size_t)kTriWalkEnd) {
        std::vector<SphereBvhNode> oct;
        std::vector<uint32_t> src;
        order_bvh_by_octant(acc.nodes, &oct, false, &src);
        std::vector<uint32_t> skip(oct.size());
        for (size_t i = 0; i < oct.size(); i++) skip[i] = oct[i].skip;
        const size_t b8 = oct.size() * 4;
        if ((rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_src8), &ctx->tri_src8_cap, b8)) ||
            (rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_skip8), &ctx->tri_skip8_cap, b8)) ||
            (rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_bvh8), &ctx->tri_bvh8_cap, oct.size() * sizeof(SphereBvhNode))) ||
            (rc = upload_raw(ctx, ctx->d_tri_src8, src.data(), b8)) ||
            (rc = upload_raw(ctx, ctx->d_tri_skip8, skip.data(), b8)))
            return rc;
        ctx->tri_octants_built = true;
    }
    // depth levels for the device refit (preorder: a node precedes its children)
    std::vector<uint32_t> depth(acc.nodes.size(), 0);
    uint32_t max_depth = 0;
    for (size_t i = 0; i < acc.nodes.size(); i++) {
        max_depth = std::max(max_depth, depth[i]);
        if (acc.nodes[i].leaf == kSphereBvhInternal) {
            depth[i + 1] = depth[i] + 1;
            depth[acc.nodes[i + 1].skip] = depth[i] + 1;
        }
    }
    std::vector<uint32_t> off(max_depth + 2, 0), order(acc.nodes.size());
    for (uint32_t d : depth) off[max_depth - d + 1]++;  // deepest level first
    for (size_t l = 1; l < off.size(); l++) off[l] += off[l - 1];
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (size_t i = 0; i < acc.nodes.size(); i++) order[fill[max_depth - depth[i]]++] = (uint32_t)i;
    if ((rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_order), &ctx->tri_order_cap, order.size() * 4)) ||
        (rc = ensure(reinterpret_cast<void**>(&ctx->d_tri_level_off), &ctx->tri_level_cap, off.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_tri_order, order.data(), order.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_tri_level_off, off.data(), off.size() * 4)) ||
        (rc = upload_raw(ctx, ctx->d_tri_extent, &acc.extent, 4)))
        return rc;
    ctx->tri_levels = max_depth + 1;
    ctx->tri_dirty = false;
    ctx->tri_count_built = object_count;
    return RT_OK;
}

int upload_triangles(rt_ctx* ctx, const rt_scene_triangle* t, uint32_t n) {
    if (n == 0) return RT_OK;
    ctx->cones_dirty = true;
    ctx->ltris_dirty = true;
    void* p;
    int rc = staging(ctx, (size_t)n * sizeof(RtTriangleHot), &p);
    if (rc) return rc;
    RtTriangleHot* hot = static_cast<RtTriangleHot*>(p);
    for (uint32_t i = 0; i < n; i++) {
        const rt_scene_triangle& s = t[i];
        hot[i] = pack_triangle(s.a, s.edge_ab, s.edge_ac, s.calc_normal, s.face_normal);
    }
    if ((rc = staged_copy(ctx, ctx->d_tri, (size_t)n * sizeof(RtTriangleHot))) ||
        (rc = staging(ctx, (size_t)n * 32, &p)))
        return rc;
    float4* b = static_cast<float4*>(p);
    for (uint32_t i = 0; i < n; i++) {
        const rt_scene_triangle& s = t[i];
        b[2 * i] = make_float4(s.min_bounds[0], s.min_bounds[1], s.min_bounds[2], 0.f);
        b[2 * i + 1] = make_float4(s.max_bounds[0], s.max_bounds[1], s.max_bounds[2], 0.f);
    }
    return staged_copy(ctx, ctx->d_tri_bounds, (size_t)n * 32);
}

// Index ranges the kernel walks must lie inside the buffers (the reference's
// fixed-size WGSL arrays would clamp; here they are rejected up front).
int validate_ranges(rt_ctx* ctx) {
    for (size_t i = 0; i < ctx->h_obj.size(); i++) {
        const rt_object_info& o = ctx->h_obj[i];
        if ((uint64_t)o.first_sub_object_index + o.sub_object_count > ctx->cap_sub)
            return fail(ctx, RT_E_INVALID, "object " + std::to_string(i) + " sub-object range exceeds sub_object_count");
    }
    for (size_t i = 0; i < ctx->h_sub.size(); i++) {
        const rt_sub_object_info& s = ctx->h_sub[i];
        if (s.triangle_count != 0 && (uint64_t)s.first_triangle_index + s.triangle_count > ctx->cap_tri)
            return fail(ctx, RT_E_INVALID, "sub-object " + std::to_string(i) + " triangle range exceeds triangle_count");
    }
    return RT_OK;
}

int check_params(rt_ctx* ctx, const rt_params* p) {
    if (!p) return fail(ctx, RT_E_INVALID, "params is NULL");
    if (p->screen_width != ctx->width)
        return fail(ctx, RT_E_INVALID, "params.screen_width must equal the framebuffer width");
    if (p->sphere_count > ctx->cap_sph) return fail(ctx, RT_E_INVALID, "params.sphere_count exceeds sphere buffer");
    if (p->object_count > ctx->cap_obj) return fail(ctx, RT_E_INVALID, "params.object_count exceeds object buffer");
    return RT_OK;
}

template <typename T>
int dev_alloc(rt_ctx* ctx, T** p, size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;  // keep every binding a valid pointer
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), bytes);
    if (e != hipSuccess) return fail(ctx, RT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    e = hipMemsetAsync(*p, 0, bytes, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "hipMemsetAsync", e);
    ctx->primary_dirty = true;
    return RT_OK;
}

// A device buffer of at least `bytes`, reallocated (after the streams drain) when smaller.
int grow_buffer(rt_ctx* ctx, void** p, size_t* cap, size_t bytes) {
    if (*p && *cap >= bytes) return RT_OK;
    RT_HIP(ctx, join_aux(ctx));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (*p) RT_HIP(ctx, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const size_t alloc = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(p, alloc);
    if (e != hipSuccess) return fail(ctx, RT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    *cap = alloc;
    return RT_OK;
}

int collect_timing(rt_ctx* ctx) {
    if (ctx->clock_pending.empty()) return RT_OK;
    RT_HIP(ctx, join_aux(ctx));
    std::vector<unsigned long long> c(kClockWords * (size_t)kClockSlots);
    RT_HIP(ctx, hipMemcpyAsync(c.data(), ctx->d_clock, c.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t slot : ctx->clock_pending) {
        const unsigned long long* w = c.data() + kClockWords * (size_t)slot;
        const unsigned long long t0 = ~w[0], t1 = w[1];
        if (w[0] != 0 && t1 >= t0) {  // else no workgroup ran
            const float ms = (float)((double)(t1 - t0) / ctx->wall_khz);
            ctx->total_ms += ms;
            ctx->n_timed += 1;
            ctx->last_ms = ms;
        }
        const unsigned long long r0 = ~w[2], r1 = w[3];
        if (w[2] != 0 && r1 >= r0) {  // the batch's resolve pass
            ctx->resolve_total_ms += (double)(r1 - r0) / ctx->wall_khz;
            ctx->n_resolve_timed += 1;
        }
    }
    ctx->clock_pending.clear();
    // the slots start the next launches at zero (the kernels atomicMax into them): cleared
    // here, off the launch path, instead of by a memset ahead of every timed launch
    RT_HIP(ctx, hipMemsetAsync(ctx->d_clock, 0, c.size() * 8, ctx->stream));
    ctx->primary_dirty = true;  // an auxiliary-stream batch waits for it
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

#ifndef RT_BUILD_HASH
#define RT_BUILD_HASH "unknown"
#endif
const char* rt_build_hash(void) { return RT_BUILD_HASH; }

const char* rt_last_error(const rt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int rt_srgb_table(float out[256]) {
    if (!out) return RT_E_INVALID;
    srgb_table(out);
    return RT_OK;
}

int rt_create(const rt_create_info* info, rt_ctx** out_ctx) {
    g_create_error.clear();
    if (!info || !out_ctx) return fail(nullptr, RT_E_INVALID, "rt_create: NULL argument");
    *out_ctx = nullptr;
    if (info->width == 0 || info->height == 0) return fail(nullptr, RT_E_INVALID, "width and height must be > 0");
    if (info->world_size == 0 || info->rank >= info->world_size)
        return fail(nullptr, RT_E_INVALID, "rank must be < world_size (world_size >= 1)");
    const uint64_t n_pixels = (uint64_t)info->width * info->height;
    if (n_pixels > 0xffffffffull) return fail(nullptr, RT_E_INVALID, "pixel index must fit in u32 (:148)");
    if (!info->camera_rays) return fail(nullptr, RT_E_INVALID, "camera_rays is NULL");
    if ((info->material_count && !info->materials) || (info->sphere_count && !info->spheres) ||
        (info->triangle_count && !info->triangles) || (info->object_count && !info->objects) ||
        (info->sub_object_count && !info->sub_objects))
        return fail(nullptr, RT_E_INVALID, "NULL scene array with a non-zero count");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0)
        return fail(nullptr, RT_E_NODEVICE, "no HIP device available");
    if (info->device < 0 || info->device >= n_dev) return fail(nullptr, RT_E_NODEVICE, "device ordinal out of range");

    rt_ctx* ctx = new (std::nothrow) rt_ctx();
    if (!ctx) return fail(nullptr, RT_E_NOMEM, "out of host memory");
    auto bail = [&](int rc) {
        g_create_error = ctx->err;
        rt_destroy(ctx);
        return rc;
    };
    ctx->device = info->device;
    ctx->width = info->width;
    ctx->height = info->height;
    ctx->n_pixels = n_pixels;
    ctx->rank = info->rank;
    ctx->world = info->world_size;
    ctx->tiles_x = (info->width + 7) / 8;
    ctx->tiles_y = (info->height + 7) / 8;
    ctx->owned_tiles = owned_tile_count(ctx->tiles_x * ctx->tiles_y, ctx->rank, ctx->world);
    ctx->camera = info->camera;
    ctx->cap_mat = info->material_count;
    ctx->cap_sph = info->sphere_count;
    ctx->cap_tri = info->triangle_count;
    ctx->cap_obj = info->object_count;
    ctx->cap_sub = info->sub_object_count;
    ctx->n_mat_dev = info->material_count ? info->material_count : 1;
    ctx->n_tri_dev = info->triangle_count ? info->triangle_count : 1;
    ctx->n_sub_dev = info->sub_object_count ? info->sub_object_count : 1;
    ctx->h_obj.assign(info->objects, info->objects + info->object_count);
    ctx->h_sph.resize(info->sphere_count);
    ctx->h_sub.assign(info->sub_objects, info->sub_objects + info->sub_object_count);

    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return bail(hip_fail(ctx, "hipSetDevice", e));
    {
        int n_cu = 0;
        e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device);
        if (e != hipSuccess) return bail(hip_fail(ctx, "hipDeviceGetAttribute", e));
        ctx->n_cu = n_cu;
        // the batch buffers' share of device memory: an eighth of the device
        size_t free_b = 0, total_b = 0;
        e = hipMemGetInfo(&free_b, &total_b);
        if (e != hipSuccess) return bail(hip_fail(ctx, "hipMemGetInfo", e));
        ctx->batch_budget = total_b / 8;
    }
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(hip_fail(ctx, "hipStreamCreate", e));
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) == hipSuccess && khz > 0)
            ctx->wall_khz = (double)khz;
    }
    e = hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(hip_fail(ctx, "hipStreamCreate (aux)", e));
    for (hipEvent_t* ev : {&ctx->staging_done, &ctx->ev_resolved[0], &ctx->ev_resolved[1], &ctx->ev_aux_done,
                           &ctx->ev_primary}) {
        e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
        if (e != hipSuccess) return bail(hip_fail(ctx, "hipEventCreate", e));
    }

    int rc;
    if ((rc = check_params(ctx, &info->params))) return bail(rc);
    if ((rc = validate_ranges(ctx))) return bail(rc);
    ctx->params = info->params;
    ctx->k = 1;  // src/renderer.rs:96

    if ((rc = dev_alloc(ctx, &ctx->d_rays, n_pixels)) || (rc = dev_alloc(ctx, &ctx->d_accum, n_pixels)) ||
        (rc = dev_alloc(ctx, &ctx->d_out, n_pixels)) || (rc = dev_alloc(ctx, &ctx->d_counter, kCounterWords)) ||
        (rc = dev_alloc(ctx, &ctx->d_queue, 4 * kQueueStripesMax * kQueueStride)) ||  // 2 streams x 2 halves
        (rc = dev_alloc(ctx, &ctx->d_slot_sph, 4 * (size_t)info->sphere_count + 4)) ||  // padded groups
        (rc = dev_alloc(ctx, &ctx->d_slot_orig, 4 * (size_t)info->sphere_count + 4)) ||
        (rc = dev_alloc(ctx, &ctx->d_sph_mat, info->sphere_count)) ||
        (rc = dev_alloc(ctx, &ctx->d_bvh, 16 * (size_t)info->sphere_count + 8)) ||  // 8 ordered layouts
        (rc = dev_alloc(ctx, &ctx->d_mat, ctx->n_mat_dev)) || (rc = dev_alloc(ctx, &ctx->d_obj, info->object_count)) ||
        (rc = dev_alloc(ctx, &ctx->d_sub, ctx->n_sub_dev)) || (rc = dev_alloc(ctx, &ctx->d_tri, ctx->n_tri_dev)) ||
        (rc = dev_alloc(ctx, &ctx->d_tri_bounds, 2 * (size_t)ctx->n_tri_dev)) ||
        (rc = dev_alloc(ctx, &ctx->d_tri_extent, 1)) || (rc = dev_alloc(ctx, &ctx->d_stream, 2)) ||
        (rc = dev_alloc(ctx, &ctx->d_srgb, 256)) || (rc = dev_alloc(ctx, &ctx->d_tex, 1)) ||
        (rc = dev_alloc(ctx, &ctx->d_env, 1)))
        return bail(rc);
    ctx->tex_w = ctx->tex_h = ctx->tex_layers = 1;  // a black 1x1 placeholder until textures arrive
    ctx->env_w = ctx->env_h = 1;

    if ((rc = upload_raw(ctx, ctx->d_rays, info->camera_rays, n_pixels * 16)) ||
        (rc = upload_raw(ctx, ctx->d_mat, info->materials, (size_t)info->material_count * 32)) ||
        (rc = upload_spheres(ctx, info->spheres, info->sphere_count)) ||
        (rc = upload_triangles(ctx, info->triangles, info->triangle_count)) ||
        (rc = upload_raw(ctx, ctx->d_obj, info->objects, (size_t)info->object_count * 48)) ||
        (rc = upload_raw(ctx, ctx->d_sub, info->sub_objects, (size_t)info->sub_object_count * 32)))
        return bail(rc);
    float lut[256];
    srgb_table(lut);
    if ((rc = upload_raw(ctx, ctx->d_srgb, lut, sizeof(lut)))) return bail(rc);
    e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return bail(hip_fail(ctx, "hipStreamSynchronize", e));
    ctx->staging_busy = false;
    *out_ctx = ctx;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)flush_frames(ctx);  // queued frames were submitted: they run before teardown
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->aux_stream) (void)hipStreamSynchronize(ctx->aux_stream);
    void* bufs[] = {ctx->d_rays, ctx->d_accum, ctx->d_out, ctx->d_counter, ctx->d_queue, ctx->d_slot_sph,
                    ctx->d_slot_orig, ctx->d_bvh, ctx->d_sph_mat, ctx->d_tri_bvh, ctx->d_tri_prims,
                    ctx->d_mat,  ctx->d_obj,   ctx->d_sub, ctx->d_tri,     ctx->d_tex,     ctx->d_env,
                    ctx->d_srgb, ctx->d_tri_extent, ctx->d_tri_order, ctx->d_tri_level_off, ctx->d_model,
                    ctx->d_tri_object, ctx->d_sub_object, ctx->d_object_tris, ctx->d_place, ctx->d_tri_bounds,
                    ctx->d_tile_sched[0], ctx->d_tile_sched[1], ctx->d_frame_light[0], ctx->d_frame_light[1],
                    ctx->d_clock, ctx->d_stream, ctx->d_primary[0], ctx->d_primary[1], ctx->d_tri_qnodes,
                    ctx->d_tri_qgrid, ctx->d_tri_src8, ctx->d_tri_skip8, ctx->d_tri_bvh8, ctx->d_tri_lcert,
                    ctx->d_tri_ltris, ctx->d_brute_paths, ctx->d_brute_queue, ctx->d_brute_counts};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    for (hipEvent_t ev : {ctx->staging_done, ctx->ev_resolved[0], ctx->ev_resolved[1], ctx->ev_aux_done,
                          ctx->ev_primary})
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->aux_stream) (void)hipStreamDestroy(ctx->aux_stream);
    delete ctx;
}

static int dispatch_frames(rt_ctx* ctx, uint32_t bounces, uint32_t frames);

// Frame batching (rt_set_frame_batch): rt_compute_frame queues frames and one
// launch renders the whole batch (each pixel's frames back to back on one lane,
// every frame's accumulation and output written). The batch is launched when it
// is full and before anything else touches the context, so every other entry
// point sees exactly the state the sequence of single-frame dispatches leaves.
static int flush_frames(rt_ctx* ctx) {
    if (ctx->pending_frames == 0) return RT_OK;
    const uint32_t n = ctx->pending_frames;
    ctx->pending_frames = 0;
    return dispatch_frames(ctx, ctx->pending_bounces, n);
}

#define RT_ENTER_NOFLUSH(ctx)                                       \
    do {                                                            \
        if (!(ctx)) return RT_E_INVALID;                            \
        (ctx)->err.clear();                                         \
        hipError_t e0_ = hipSetDevice((ctx)->device);               \
        if (e0_ != hipSuccess) return hip_fail(ctx, "hipSetDevice", e0_); \
    } while (0)

// Every entry point but rt_compute_frame: launch the queued frames, order the
// primary stream after the auxiliary one, and note that primary-stream work may
// follow (a later overlapped batch then waits for it).
#define RT_ENTER(ctx)                                                   \
    do {                                                                \
        RT_ENTER_NOFLUSH(ctx);                                          \
        const int rcf_ = flush_frames(ctx);                             \
        if (rcf_ != RT_OK) return rcf_;                                 \
        const hipError_t ej_ = join_aux(ctx);                           \
        if (ej_ != hipSuccess) return hip_fail(ctx, "join_aux", ej_);   \
        (ctx)->primary_dirty = true;                                    \
    } while (0)

int rt_upload_textures(rt_ctx* ctx, const uint8_t* rgba8, uint32_t width, uint32_t height, uint32_t layers) {
    RT_ENTER(ctx);
    if (!rgba8 || width == 0 || height == 0 || layers == 0)
        return fail(ctx, RT_E_INVALID, "textures: need non-empty RGBA8 data");
    const size_t texels = (size_t)width * height * layers;
    if (texels != (size_t)ctx->tex_w * ctx->tex_h * ctx->tex_layers || !ctx->d_tex) {
        RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->d_tex) RT_HIP(ctx, hipFree(ctx->d_tex));
        ctx->d_tex = nullptr;
        RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_tex), texels * 4));
    }
    ctx->tex_w = width;
    ctx->tex_h = height;
    ctx->tex_layers = layers;
    return upload_raw(ctx, ctx->d_tex, rgba8, texels * 4);
}

int rt_upload_env_map(rt_ctx* ctx, const uint8_t* rgba8, uint32_t width, uint32_t height) {
    RT_ENTER(ctx);
    if (!rgba8 || width == 0 || height == 0) return fail(ctx, RT_E_INVALID, "env map: need non-empty RGBA8 data");
    const size_t texels = (size_t)width * height;
    if (texels != (size_t)ctx->env_w * ctx->env_h || !ctx->d_env) {
        RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->d_env) RT_HIP(ctx, hipFree(ctx->d_env));
        ctx->d_env = nullptr;
        RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_env), texels * 4));
    }
    ctx->env_w = width;
    ctx->env_h = height;
    // A map whose rows (columns) are each one colour returns the same texel for
    // any u (v): the kernel then skips that coordinate's atan2 (asin).
    const uint32_t* t = reinterpret_cast<const uint32_t*>(rgba8);
    bool rows = true, cols = true;
    for (size_t y = 0; y < height && rows; y++)
        for (size_t x = 1; x < width; x++)
            if (t[y * width + x] != t[y * width]) {
                rows = false;
                break;
            }
    for (size_t y = 1; y < height && cols; y++)
        for (size_t x = 0; x < width; x++)
            if (t[y * width + x] != t[x]) {
                cols = false;
                break;
            }
    ctx->env_uniform = (rows ? 1u : 0u) | (cols ? 2u : 0u);
    return upload_raw(ctx, ctx->d_env, rgba8, texels * 4);
}

int rt_update_params(rt_ctx* ctx, const rt_params* params) {
    RT_ENTER(ctx);
    int rc = check_params(ctx, params);
    if (rc) return rc;
    ctx->params = *params;
    return RT_OK;
}

int rt_reset_accumulation(rt_ctx* ctx, const rt_params* params) {
    RT_ENTER(ctx);
    int rc = check_params(ctx, params);
    if (rc) return rc;
    RT_HIP(ctx, hipMemsetAsync(ctx->d_accum, 0, ctx->n_pixels * 16, ctx->stream));
    ctx->params = *params;
    ctx->k = params->accumulation_index;
    return RT_OK;
}

int rt_update_ray_directions(rt_ctx* ctx, const rt_ray* rays, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !rays) return fail(ctx, RT_E_INVALID, "rays is NULL");
    if (count > ctx->n_pixels) return fail(ctx, RT_E_CAPACITY, "more rays than pixels");
    ctx->gen_rays = false;
    return upload_raw(ctx, ctx->d_rays, rays, (size_t)count * 16);
}

int rt_update_camera_matrices(rt_ctx* ctx, const float inverse_projection[16], const float inverse_view[16]) {
    RT_ENTER(ctx);
    if (!inverse_projection || !inverse_view) return fail(ctx, RT_E_INVALID, "matrix is NULL");
    std::memcpy(ctx->inv_proj, inverse_projection, sizeof(ctx->inv_proj));
    std::memcpy(ctx->inv_view, inverse_view, sizeof(ctx->inv_view));
    ctx->gen_rays = true;
    return RT_OK;
}

int rt_update_camera(rt_ctx* ctx, const rt_ray_camera* camera) {
    RT_ENTER(ctx);
    if (!camera) return fail(ctx, RT_E_INVALID, "camera is NULL");
    ctx->camera = *camera;  // passed by value to the next launch
    return RT_OK;
}

int rt_update_spheres(rt_ctx* ctx, const rt_scene_sphere* spheres, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !spheres) return fail(ctx, RT_E_INVALID, "spheres is NULL");
    if (count > ctx->cap_sph) return fail(ctx, RT_E_CAPACITY, "more spheres than the buffer holds");
    return upload_spheres(ctx, spheres, count);
}

int rt_update_triangles(rt_ctx* ctx, const rt_scene_triangle* triangles, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !triangles) return fail(ctx, RT_E_INVALID, "triangles is NULL");
    if (count > ctx->cap_tri) return fail(ctx, RT_E_CAPACITY, "more triangles than the buffer holds");
    return upload_triangles(ctx, triangles, count);
}

int rt_update_object_info(rt_ctx* ctx, const rt_object_info* objects, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !objects) return fail(ctx, RT_E_INVALID, "objects is NULL");
    if (count > ctx->cap_obj) return fail(ctx, RT_E_CAPACITY, "more objects than the buffer holds");
    int rc0 = sync_host_geometry(ctx);
    if (rc0) return rc0;
    std::vector<rt_object_info> saved = ctx->h_obj;
    std::copy(objects, objects + count, ctx->h_obj.begin());
    int rc = validate_ranges(ctx);
    if (rc) {
        ctx->h_obj.swap(saved);
        return rc;
    }
    // the accelerator culls with the object boxes and walks the sub-object
    // ranges; the device edit path's maps follow the ranges. A change of the
    // other fields (material_index) invalidates neither.
    bool boxes = false, ranges = false;
    for (uint32_t i = 0; i < count; i++) {
        const rt_object_info &a = saved[i], &b = objects[i];
        boxes |= std::memcmp(a.min_bounds, b.min_bounds, 12) != 0 || std::memcmp(a.max_bounds, b.max_bounds, 12) != 0;
        ranges |= a.first_sub_object_index != b.first_sub_object_index || a.sub_object_count != b.sub_object_count;
    }
    if (boxes || ranges) ctx->tri_dirty = true;
    if (ranges) ctx->models_valid = false;
    return upload_raw(ctx, ctx->d_obj, objects, (size_t)count * 48);
}

int rt_update_sub_object_info(rt_ctx* ctx, const rt_sub_object_info* sub_objects, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !sub_objects) return fail(ctx, RT_E_INVALID, "sub_objects is NULL");
    if (count > ctx->cap_sub) return fail(ctx, RT_E_CAPACITY, "more sub-objects than the buffer holds");
    int rc0 = sync_host_geometry(ctx);
    if (rc0) return rc0;
    std::vector<rt_sub_object_info> saved = ctx->h_sub;
    std::copy(sub_objects, sub_objects + count, ctx->h_sub.begin());
    int rc = validate_ranges(ctx);
    if (rc) {
        ctx->h_sub.swap(saved);
        return rc;
    }
    for (uint32_t i = 0; i < count; i++)
        if (saved[i].first_triangle_index != sub_objects[i].first_triangle_index ||
            saved[i].triangle_count != sub_objects[i].triangle_count)
            ctx->models_valid = false;  // the device edit path's triangle maps are stale
    ctx->tri_dirty = true;
    return upload_raw(ctx, ctx->d_sub, sub_objects, (size_t)count * 32);
}

int rt_update_materials(rt_ctx* ctx, const rt_scene_material* materials, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !materials) return fail(ctx, RT_E_INVALID, "materials is NULL");
    if (count > ctx->cap_mat) return fail(ctx, RT_E_CAPACITY, "more materials than the buffer holds");
    return upload_raw(ctx, ctx->d_mat, materials, (size_t)count * 32);
}

static int dispatch_frames(rt_ctx* ctx, uint32_t bounces, uint32_t frames);

int rt_dispatch(rt_ctx* ctx, uint32_t bounces) {
    RT_ENTER(ctx);
    return dispatch_frames(ctx, bounces, 1);
}

static int dispatch_batch(rt_ctx* ctx, uint32_t bounces, uint32_t frames);

// Renders `frames` frames starting at Params.accumulation_index: one launch (dispatch_batch),
// or, when the batch's buffers -- the frame lights and the primary records, 32 B per owned
// pixel, frame and sample each -- would outgrow the batch budget (an eighth of the device's
// memory by default), consecutive launches of as many frames as fit, which render the same
// bits: frames are independent but for the accumulation, which every launch adds to in order.
static int dispatch_frames(rt_ctx* ctx, uint32_t bounces, uint32_t frames) {
    const rt_params& p = ctx->params;
    const uint64_t samples = std::max<uint32_t>(1u, p.accumulate == 1u ? p.compute_per_frame : 1u);
    const uint64_t per_frame = (uint64_t)ctx->owned_tiles * 64u * samples * 2u * 2u * sizeof(float4);
    const uint64_t fit = std::max<uint64_t>(1u, ctx->batch_budget / std::max<uint64_t>(1u, per_frame));
    if (frames <= fit) return dispatch_batch(ctx, bounces, frames);
    const uint32_t k0 = ctx->params.accumulation_index;
    int rc = RT_OK;
    for (uint32_t done = 0; done < frames && rc == RT_OK;) {
        const uint32_t n = (uint32_t)std::min<uint64_t>(fit, frames - done);
        if (p.accumulate == 1u) ctx->params.accumulation_index = k0 + done;
        rc = dispatch_batch(ctx, bounces, n);
        done += n;
    }
    ctx->params.accumulation_index = k0;  // the batch's Params, as one launch leaves them
    return rc;
}

// One launch rendering `frames` frames starting at Params.accumulation_index.
static int dispatch_batch(rt_ctx* ctx, uint32_t bounces, uint32_t frames) {
    const rt_params& p = ctx->params;
    {
        int rc = refresh_sphere_slots(ctx, p.sphere_count, p.object_count == 0);
        if (rc) return rc;
        rc = refresh_tri_accel(ctx, p.object_count);
        if (rc) return rc;
    }
    KernelArgs ka{};
    ka.camera_rays = ctx->d_rays;
    ka.accum = ctx->d_accum;
    ka.output = ctx->d_out;
    ka.ray_counter = ctx->d_counter;
    ka.diag = ctx->d_counter + 1;
    ka.queue_stripes = ctx->queue_stripes;  // (queue counters: per stream, set at launch)
    ka.sphere_slots = ctx->d_slot_sph;
    ka.sphere_orig = ctx->d_slot_orig;
    ka.sphere_material = ctx->d_sph_mat;
    ka.sphere_bvh = reinterpret_cast<const float4*>(ctx->d_bvh);
    ka.sphere_always = ctx->n_always;
    ka.sphere_nodes = ctx->n_nodes;
    ka.sphere_extent = ctx->sphere_extent;
    ka.sphere_rmin = ctx->sphere_rmin;
    ka.sphere_rmax = ctx->sphere_rmax;
    ka.tri_accel = (ctx->use_tri_bvh && p.object_count != 0) ? 1u : 0u;
    ka.tri_nodes = ka.tri_accel ? ctx->tri_nodes : 0u;
    ka.tri_prim_count = ka.tri_accel ? ctx->tri_prim_count : 0u;
    ka.tri_extent = ctx->d_tri_extent;
    ka.tri_bvh = reinterpret_cast<const float4*>(ctx->d_tri_bvh);
    ka.tri_prims = reinterpret_cast<const uint4*>(ctx->d_tri_prims);
    ka.materials = ctx->d_mat;
    ka.objects = ctx->d_obj;
    ka.sub_objects = ctx->d_sub;
    ka.triangles = ctx->d_tri;
    ka.textures = ctx->d_tex;
    ka.env = ctx->d_env;
    ka.srgb = ctx->d_srgb;
    ka.camera_origin[0] = ctx->camera.origin[0];
    ka.camera_origin[1] = ctx->camera.origin[1];
    ka.camera_origin[2] = ctx->camera.origin[2];
    ka.width = ctx->width;
    ka.accumulation_index = p.accumulation_index;
    ka.accumulate = p.accumulate;
    ka.sphere_count = p.sphere_count;
    ka.sphere_slot_count = ctx->n_slots;
    ka.object_count = p.object_count;
    ka.compute_per_frame = p.compute_per_frame;
    ka.texture_width = p.texture_width;
    ka.texture_height = p.texture_height;
    ka.env_map_width = p.env_map_width;
    ka.env_map_height = p.env_map_height;
    ka.material_count = ctx->n_mat_dev;
    ka.sub_object_count = ctx->n_sub_dev;
    ka.triangle_count = ctx->n_tri_dev;
    ka.tex_w = ctx->tex_w;
    ka.tex_h = ctx->tex_h;
    ka.tex_layers = ctx->tex_layers;
    ka.env_w = ctx->env_w;
    ka.env_h = ctx->env_h;
    ka.env_uniform = ctx->env_uniform;
    ka.height = ctx->height;
    ka.gen_rays = ctx->gen_rays ? 1u : 0u;
    ka.aspect = (float)ctx->width / (float)ctx->height;  // src/camera.rs:142
    std::memcpy(ka.inv_proj, ctx->inv_proj, sizeof(ka.inv_proj));
    std::memcpy(ka.inv_view, ctx->inv_view, sizeof(ka.inv_view));
    ka.bounces = bounces;
    ka.tiles_x = ctx->tiles_x;
    ka.owned_tiles = ctx->owned_tiles;
    ka.rank = ctx->rank;
    ka.world_size = ctx->world;
    ka.drain_threshold = ctx->drain_threshold;
    ka.drain_min_steps = ctx->drain_min_steps;
    ka.frames = frames;
    // Frame-parallel batch: one queue unit per (frame, tile), lights resolved in order
    // by rt_resolve_frames_kernel (accumulating renders; non-accumulating frames are
    // all the same frame and keep the per-lane sequence).
    const uint64_t owned_px = (uint64_t)ctx->owned_tiles * 64u;
    const bool frame_par = frames > 1 && p.accumulate == 1u && ctx->frame_parallel &&
                           (uint64_t)frames * p.compute_per_frame <= kMaxParallelLights && p.compute_per_frame > 0;
    ka.frame_light = nullptr;
    ka.queue_units = ctx->owned_tiles;
    if (frame_par) {
        const size_t need = (size_t)owned_px * frames * p.compute_per_frame;
        if (need > ctx->frame_light_cap) {
            // sized for the configured batch too, so a short first batch (a warmup)
            // does not leave a reallocation for a later, timed launch; two buffers,
            // one per batch parity (overlapped batches), within the batch budget
            const size_t want = std::max<size_t>(
                need, std::min<size_t>(ctx->batch_budget / (2 * sizeof(float4)),
                                       (size_t)owned_px * std::min<uint64_t>((uint64_t)ctx->frame_batch *
                                                                                 p.compute_per_frame,
                                                                             kMaxParallelLights)));
            RT_HIP(ctx, join_aux(ctx));
            RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            for (float4*& b : ctx->d_frame_light) {
                if (b) RT_HIP(ctx, hipFree(b));
                b = nullptr;
            }
            ctx->frame_light_cap = 0;
            for (float4*& b : ctx->d_frame_light) {
                const hipError_t ea = hipMalloc(reinterpret_cast<void**>(&b), want * sizeof(float4));
                if (ea != hipSuccess) return fail(ctx, RT_E_NOMEM, std::string("frame lights: ") + hipGetErrorString(ea));
            }
            ctx->frame_light_cap = want;
        }
        ka.queue_units = ctx->owned_tiles * frames;
        ka.unit_tile_major = ctx->unit_tile_major ? 1u : 0u;
    }

    // dynamic LDS carve-up: sphere slots | materials | objects | slot->orig | sphere materials | BVH | srgb
    auto al16 = [](size_t x) { return (x + 15) & ~size_t(15); };
    const bool tris = p.object_count != 0;  // else the sphere-only kernels
    size_t mode1_bytes = 0, mode2_bytes = 0;
    // lays out the LDS image for `layouts` sphere BVH layouts and returns the LDS mode it fits
    auto carve = [&](uint32_t layouts, size_t mode1_budget) -> int {
        size_t off = al16((size_t)ctx->n_slots * 16);
        ka.lds_mat_offset = (uint32_t)off;
        off = al16(off + (size_t)ctx->n_mat_dev * sizeof(RtMaterial));
        ka.lds_mat_aux_offset = (uint32_t)off;
        off = al16(off + (size_t)ctx->n_mat_dev * 32);
        ka.lds_obj_offset = (uint32_t)off;
        off = al16(off + (size_t)p.object_count * sizeof(RtObject));
        ka.lds_orig_offset = (uint32_t)off;
        off = al16(off + (size_t)ctx->n_slots * 4);
        ka.lds_smat_offset = (uint32_t)off;
        off = al16(off + (size_t)p.sphere_count * 4);
        ka.lds_nodes_offset = (uint32_t)off;
        off = al16(off + (size_t)layouts * ctx->n_nodes * sizeof(SphereBvhNode));
        mode1_bytes = off + kLdsTailBytes;
        ka.lds_tri_nodes_offset = (uint32_t)off;
        off = al16(off + (size_t)ka.tri_nodes * sizeof(SphereBvhNode));
        ka.lds_tri_prims_offset = (uint32_t)off;
        off = al16(off + (size_t)ka.tri_prim_count * sizeof(SubObjectPrim));
        // the sub-object records the leaves read, when they fit the mode-2 budget too
        // (one dependent global load less per leaf test; tuning "stage_subs" 0 switches it off)
        ka.lds_sub_offset = 0;
        if (ctx->stage_subs && ka.sub_object_count != 0) {
            const size_t with = al16(off + (size_t)ka.sub_object_count * sizeof(RtSubObject));
            if (with + kLdsTailBytes <= kLdsAccelBudget) {
                ka.lds_sub_offset = (uint32_t)off;
                off = with;
            }
        }
        mode2_bytes = off + kLdsTailBytes;
        if (ctx->force_global_scene) return 0;
        if (ka.tri_accel && ka.tri_nodes != 0 && mode2_bytes <= kLdsAccelBudget && ctx->max_lds_mode >= 2)
            return 2;
        if (mode1_bytes <= mode1_budget && ctx->max_lds_mode >= 1) return 1;
        return 0;
    };
    // Direction-ordered sphere BVH layouts (order_bvh_by_octant) when all eight
    // fit the LDS mode that one layout gets (up to the mode-2 budget, in fewer,
    // larger workgroups); otherwise layout 0 alone.
    int mode = carve(1, kLdsSceneBudget);
    uint32_t layouts = 1;
    if (ctx->sphere_octants && ctx->n_nodes != 0) {
        if (carve(8, kLdsAccelBudget) == mode)
            layouts = 8;
        else
            carve(1, kLdsSceneBudget);
    }
    if (ctx->brute) {
        // the reference's sweeps as a wavefront (rt_brute_wf_kernel): the mode-1 scene image,
        // then the sub-object tiles (mode 1) or the hit lists (mode 2: the records through the
        // scalar cache; a scene without triangles has no records to stream and sweeps its
        // spheres in the LDS-tiled kernel); every pass (frame, sample) in order, one launch per
        // bounce level
        carve(1, kLdsSceneBudget);
        ka.lds_srgb_offset = (uint32_t)(mode1_bytes - kLdsTailBytes);
        ka.lds_stack_offset = (uint32_t)al16(mode1_bytes);
        const uint32_t samples = ka.accumulate == 1u ? ka.compute_per_frame : 1u;
        const uint64_t passes = (uint64_t)frames * samples;
        const bool scalar_stream = tris && ctx->brute == 2;
        const size_t lds = ka.lds_stack_offset + rt_brute_wf_tile_bytes(scalar_stream);
        int dev = 0, max_optin = 0;
        RT_HIP(ctx, hipGetDevice(&dev));
        RT_HIP(ctx, hipDeviceGetAttribute(&max_optin, hipDeviceAttributeSharedMemPerBlockOptin, dev));
        if (lds > (size_t)max_optin - 256)
            return fail(ctx, RT_E_CAPACITY, "brute-force mode: spheres, materials and objects must fit in LDS");
        ka.sphere_octant_stride = 0;
        ka.sphere_boxes_ordered = 0;
        ka.stream_bytes = ctx->d_stream;
        ka.l2_stream_bytes = ctx->d_stream + 1;
        ka.frame_light = nullptr;
        RT_HIP(ctx, join_aux(ctx));
        ka.launch_clock = nullptr;
        if (ctx->timing) {
            if (ctx->clock_pending.size() >= kClockSlots) {
                const int rc = collect_timing(ctx);
                if (rc) return rc;
            }
            if (!ctx->d_clock) {
                const int rc = dev_alloc(ctx, &ctx->d_clock, kClockWords * (size_t)kClockSlots);
                if (rc) return rc;
            }
            const uint32_t slot = ctx->clock_next;
            ctx->clock_next = (ctx->clock_next + 1) % kClockSlots;
            ka.launch_clock = ctx->d_clock + kClockWords * (size_t)slot;  // zero: dev_alloc / collect_timing
            ctx->clock_pending.push_back(slot);
        }
        const size_t n_slots = (size_t)ctx->owned_tiles * 64u;
        // per pass one counter per bounce level: the entries of each level's queue
        ka.brute_levels = std::max(1u, bounces) + 1u;
        const size_t n_counts = (size_t)passes * ka.brute_levels;
        int rc;
        if ((rc = grow_buffer(ctx, reinterpret_cast<void**>(&ctx->d_brute_paths), &ctx->brute_paths_cap,
                              4 * n_slots * sizeof(float4))) ||
            (rc = grow_buffer(ctx, reinterpret_cast<void**>(&ctx->d_brute_queue), &ctx->brute_queue_cap,
                              2 * n_slots * sizeof(uint32_t))) ||
            (rc = grow_buffer(ctx, reinterpret_cast<void**>(&ctx->d_brute_counts), &ctx->brute_counts_cap,
                              n_counts * sizeof(uint32_t))))
            return rc;
        RT_HIP(ctx, hipMemsetAsync(ctx->d_brute_counts, 0, n_counts * sizeof(uint32_t), ctx->stream));
        ka.brute_paths = ctx->d_brute_paths;
        ka.brute_queue = ctx->d_brute_queue;
        ka.brute_counts = ctx->d_brute_counts;
        // workgroups per launch: enough for every chunk of queue entries, at most 16 per CU
        const uint32_t chunks = (uint32_t)((n_slots + rt_brute_wf_chunk() - 1u) / rt_brute_wf_chunk());
        const uint32_t blocks = std::min<uint32_t>(chunks, 16u * (uint32_t)std::max<int>(1, (int)ctx->n_cu));
        for (uint64_t pass = 0; pass < passes; ++pass)
            for (uint32_t level = 0; level < std::max(1u, bounces); ++level) {
                ka.brute_pass = (uint32_t)pass;
                ka.brute_level = level;
                RT_HIP(ctx, rt_launch_brute_wf(ka, tris, scalar_stream, lds, blocks, ctx->stream));
            }
        ctx->last_blocks = blocks;
        ctx->last_passes = RT_PASS_BRUTE | (scalar_stream ? RT_PASS_BRUTE_STREAM : 0u);
        ctx->last_lds = (uint32_t)lds;
        ctx->occ_threads = 256;
        ctx->primary_dirty = true;
        return RT_OK;
    }
    ka.sphere_nodes = layouts * ctx->n_nodes;
    ka.sphere_octant_stride = layouts == 8 ? ctx->n_nodes : 0u;
    ka.sphere_boxes_ordered = (layouts == 8 && ctx->sphere_boxes_ordered && !tris) ? 1u : 0u;
    const bool certified = tris && mode <= 1 && ka.tri_accel && ctx->tri_prune_mode == 1;
    ka.trav_threshold = ctx->trav_threshold ? ctx->trav_threshold : trav_threshold_for(mode, tris, certified);
    ka.leaf_batch = ctx->leaf_batch ? ctx->leaf_batch : leaf_batch_for(mode, certified);
    // walks of the binary triangle accelerator from global memory read its direction-ordered
    // layouts (8 x tri_nodes positions, 32-B and 16-B quantized copies), else the single one
    ka.tri_qnodes = nullptr;
    ka.tri_qgrid = nullptr;
    ka.tri_octant_stride = 0;
    const bool global_walk = tris && mode <= 1 && ka.tri_accel && ka.tri_nodes != 0;
    const bool octants = global_walk && ctx->tri_octants_built;
    const bool qnodes = global_walk && ctx->use_qnodes;
    if (octants || qnodes) {
        const uint32_t n_out = octants ? 8u * ka.tri_nodes : ka.tri_nodes;
        if (qnodes && ctx->qnodes_cap < n_out) {
            RT_HIP(ctx, join_aux(ctx));
            RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->d_tri_qnodes) RT_HIP(ctx, hipFree(ctx->d_tri_qnodes));
            ctx->d_tri_qnodes = nullptr;
            ctx->qnodes_cap = 0;
            RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_tri_qnodes), (size_t)n_out * sizeof(uint4)));
            ctx->qnodes_cap = n_out;
            ctx->qnodes_dirty = true;
        }
        if (!ctx->d_tri_qgrid) RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_tri_qgrid), 2 * sizeof(float4)));
        if (ctx->qnodes_dirty || ctx->derived_octants != octants || ctx->derived_qnodes != qnodes) {
            // after the accelerator's upload or refit (primary stream)
            RT_HIP(ctx, rt_launch_quantize_tri_nodes(reinterpret_cast<const SphereBvhNode*>(ctx->d_tri_bvh),
                                                     ka.tri_nodes, octants ? ctx->d_tri_src8 : nullptr,
                                                     octants ? ctx->d_tri_skip8 : nullptr, n_out,
                                                     octants ? ctx->d_tri_bvh8 : nullptr,
                                                     qnodes ? ctx->d_tri_qnodes : nullptr, ctx->d_tri_qgrid,
                                                     ctx->stream));
            ctx->qnodes_dirty = false;
            ctx->derived_octants = octants;
            ctx->derived_qnodes = qnodes;
            ctx->primary_dirty = true;  // an auxiliary-stream batch waits for it
        }
        if (qnodes) {
            ka.tri_qnodes = ctx->d_tri_qnodes;
            ka.tri_qgrid = ctx->d_tri_qgrid;
        }
        if (octants) {
            ka.tri_bvh = reinterpret_cast<const float4*>(ctx->d_tri_bvh8);
            ka.tri_octant_stride = ka.tri_nodes;
            ka.tri_nodes = n_out;
        }
    }
    // distance pruning of the binary walk: certified (the leaf certificates,
    // rebuilt on the device after any change), or the round-3 relative slack, or none
    ka.tri_prune_mode = (tris && ka.tri_accel && ka.tri_nodes != 0) ? (uint32_t)ctx->tri_prune_mode : 0u;
    ka.tri_prune = ka.tri_prune_mode == 2u ? kTriPruneRho : 0.0f;
    ka.tri_leafcert = nullptr;
    if (ka.tri_prune_mode == 1u && ka.tri_prim_count != 0 && mode <= 1) {  // (mode 2 culls by box alone)
        const size_t bytes = (size_t)ka.tri_prim_count * sizeof(TriLeafCert);
        if (ctx->tri_lcert_cap < bytes) {  // (re)allocate: nothing may still read them
            RT_HIP(ctx, join_aux(ctx));
            RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->d_tri_lcert) RT_HIP(ctx, hipFree(ctx->d_tri_lcert));
            ctx->d_tri_lcert = nullptr;
            ctx->tri_lcert_cap = 0;
            RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_tri_lcert), bytes));
            ctx->tri_lcert_cap = bytes;
            ctx->cones_dirty = true;
        }
        if (ctx->cones_dirty) {
            RT_HIP(ctx, rt_launch_tri_leafcert(ctx->d_tri_prims, ka.tri_prim_count, ctx->d_sub, ctx->d_tri,
                                               ctx->n_tri_dev, ctx->d_tri_lcert, ctx->stream));
            ctx->cones_dirty = false;
            ctx->primary_dirty = true;  // an auxiliary-stream batch waits for it
        }
        ka.tri_leafcert = ctx->d_tri_lcert;
    }
    // cooperative leaf batches (walks from global memory): the leaves' triangle blocks
    ka.tri_leaftris = nullptr;
    const bool coop = tris && mode <= 1 && ka.tri_accel && ka.tri_nodes != 0 && ka.tri_prim_count != 0 &&
                      ctx->use_coop_leaves;
    if (coop) {
        const size_t bytes = (size_t)ka.tri_prim_count * kLeafTriWords * sizeof(uint4);
        if (ctx->tri_ltris_cap < bytes) {  // (re)allocate: nothing may still read them
            RT_HIP(ctx, join_aux(ctx));
            RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->d_tri_ltris) RT_HIP(ctx, hipFree(ctx->d_tri_ltris));
            ctx->d_tri_ltris = nullptr;
            ctx->tri_ltris_cap = 0;
            RT_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_tri_ltris), bytes));
            ctx->tri_ltris_cap = bytes;
            ctx->ltris_dirty = true;
        }
        if (ctx->ltris_dirty) {
            RT_HIP(ctx, rt_launch_tri_leaftris(ctx->d_tri_prims, ka.tri_prim_count, ctx->d_tri, ctx->n_tri_dev,
                                               ctx->d_tri_ltris, ctx->stream));
            ctx->ltris_dirty = false;
            ctx->primary_dirty = true;  // an auxiliary-stream batch waits for it
        }
        ka.tri_leaftris = ctx->d_tri_ltris;
    }
    size_t lds_bytes;
    if (mode == 2) {
        ka.lds_srgb_offset = (uint32_t)(mode2_bytes - kLdsTailBytes);
        lds_bytes = mode2_bytes;
    } else if (mode == 1) {
        ka.lds_srgb_offset = (uint32_t)(mode1_bytes - kLdsTailBytes);
        lds_bytes = mode1_bytes;
    } else {
        ka.lds_srgb_offset = 0;
        lds_bytes = kLdsTailBytes;
    }
    // per-thread LDS after the scene image: the cooperative leaf batch's per-wave scratch
    const size_t lane_pt = coop ? (size_t)kLeafBatchWaveBytes / 64u : 0u;
    // Persistent grid: as many workgroups as can be resident (never more than
    // one wave per tile); waves then pull tiles from the queue.
    if (ctx->occ_blocks_per_cu == 0 || ctx->occ_lds_bytes != lds_bytes || ctx->occ_mode != mode ||
        ctx->occ_tris != tris || ctx->occ_stack_pt != lane_pt) {
        int per_cu = 0;
        uint32_t threads = 0;
        hipError_t oe = rt_pathtrace_pick_config(mode, tris, lds_bytes, lane_pt, ctx->force_threads, ctx->waves_cap,
                                                 &threads, &per_cu);
        if (oe != hipSuccess) return hip_fail(ctx, "rt_pathtrace_pick_config (occupancy query)", oe);
        ctx->occ_blocks_per_cu = per_cu;
        ctx->occ_threads = threads;
        ctx->occ_lds_bytes = lds_bytes;
        ctx->occ_mode = mode;
        ctx->occ_tris = tris;
        ctx->occ_stack_pt = lane_pt;
    }
    // the leaf batch scratch after the scene image and its tail
    ka.lds_leafbatch_offset = (uint32_t)al16(lds_bytes);
    if (coop) lds_bytes = ka.lds_leafbatch_offset + (size_t)ctx->occ_threads * lane_pt;
    const uint32_t waves_per_block = ctx->occ_threads / 64;
    const uint64_t resident = (uint64_t)ctx->occ_blocks_per_cu * (uint64_t)(ctx->n_cu > 0 ? ctx->n_cu : 1);
    const uint64_t wanted = ((uint64_t)ka.queue_units + waves_per_block - 1) / waves_per_block;
    const uint32_t blocks = (uint32_t)(wanted < resident ? wanted : resident);
    if (blocks == 0) return RT_OK;
    // Cost-ordered schedule, when each wave takes several tiles per launch (with
    // about one tile per wave the claim order cannot shorten the drain, and the
    // sort would sit on a short launch's critical path).
    // Frame-parallel batches claim in index order: with the drain paid once per batch
    // (and overlapped) the cost order's recording and sort cost more than they save,
    // and index order keeps neighbouring tiles together (C2 -5.2%, C3 -2.7% per frame
    // measured, profiles/archive/r02_knobs); RT_BATCH_SCHEDULE=1 sorts them too (A/B switch).
    const bool sched = ctx->tile_schedule && (!frame_par || ctx->batch_schedule) &&
                       (uint64_t)ka.queue_units >= kSchedMinTilesPerWave * blocks * waves_per_block;
    // Overlapped batches: frame-parallel batches alternate between
    // the primary and the auxiliary stream. Batch i's path kernel depends on no
    // other batch (it writes its own light buffer, i % 2), so it starts on the CUs
    // that batch i-1's drain frees; only its resolve waits for batch i-1's resolve
    // (the accumulation order). Everything else stays on the primary stream.
    const int si = (frame_par && ctx->batch_overlap) ? (int)(ctx->batches & 1u) : 0;
    hipStream_t S = si ? ctx->aux_stream : ctx->stream;
    if (!frame_par) RT_HIP(ctx, join_aux(ctx));  // a plain launch follows every earlier batch
    if (si && ctx->primary_dirty) {  // primary-stream work (uploads, resets) the batch must follow
        RT_HIP(ctx, hipEventRecord(ctx->ev_primary, ctx->stream));
        RT_HIP(ctx, hipStreamWaitEvent(S, ctx->ev_primary, 0));
        ctx->primary_dirty = false;
    }
    ka.queue = ctx->d_queue + (size_t)(2 * si + ctx->queue_parity[si]) * kQueueStripesMax * kQueueStride;
    ka.queue_next = ctx->d_queue + (size_t)(2 * si + (ctx->queue_parity[si] ^ 1u)) * kQueueStripesMax * kQueueStride;
    if (frame_par) ka.frame_light = ctx->d_frame_light[ctx->batches & 1u];
    if (sched) {
        const size_t n = ctx->owned_tiles;
        uint32_t*& state = ctx->d_tile_sched[si];
        if (!state) {
            int rc = dev_alloc(ctx, &state, 4 * n + 2);
            if (rc) return rc;
            RT_HIP(ctx, hipMemsetAsync(state, 0, (4 * n + 2) * 4, ctx->stream));
            ctx->primary_dirty = true;
            if (si) {
                RT_HIP(ctx, hipEventRecord(ctx->ev_primary, ctx->stream));
                RT_HIP(ctx, hipStreamWaitEvent(S, ctx->ev_primary, 0));
            }
            ctx->sched_launches[si] = 0;
        }
        ka.sched = state;
        // orders[parity] was written by this stream's previous launch
        ka.sched_bits = (uint32_t)(ctx->sched_launches[si] & 1u);
        ka.tile_cost = ka.sched + ka.sched_bits * (size_t)n;
        ka.tile_order = ctx->sched_launches[si] ? ka.sched + (2u + ka.sched_bits) * (size_t)n : nullptr;
    }

    ka.launch_clock = nullptr;
    if (ctx->timing) {
        if (ctx->clock_pending.size() >= kClockSlots) {
            const int rc = collect_timing(ctx);
            if (rc) return rc;
        }
        if (!ctx->d_clock) {
            const int rc = dev_alloc(ctx, &ctx->d_clock, kClockWords * (size_t)kClockSlots);
            if (rc) return rc;
            if (si) {  // the zeroed slots must be in place before an aux launch
                RT_HIP(ctx, hipEventRecord(ctx->ev_primary, ctx->stream));
                RT_HIP(ctx, hipStreamWaitEvent(S, ctx->ev_primary, 0));
            }
        }
        const uint32_t slot = ctx->clock_next;
        ctx->clock_next = (ctx->clock_next + 1) % kClockSlots;
        ka.launch_clock = ctx->d_clock + kClockWords * (size_t)slot;  // zero: dev_alloc / collect_timing
        ctx->clock_pending.push_back(slot);
    }
    // Coherent primary rays: the first segment of every (frame, sample, pixel) of the launch
    // traced by rt_primary_kernel as 8x8 packets, stream-ordered before the path kernel
    // (scene image in LDS, binary triangle accelerator). By default only where the triangle
    // accelerator stays in global memory (mode 1 with triangles, C5: wall -12%); with the
    // accelerator in LDS (C3, C4) or no triangles (C2) the pass costs more wall time than it
    // takes off the path kernel (+13%, +13%, +23%: profiles/r03_i/ab_primary.jsonl)
    // (within the batch budget: a batch too large for it traces its first segments in the path kernel)
    const size_t primary_need =
        (size_t)owned_px * frames * std::max<uint32_t>(1u, p.accumulate == 1u ? p.compute_per_frame : 1u);
    const bool primary = bounces > 0 && mode >= 1 && tris && ka.compute_per_frame > 0 &&
                         (ctx->primary_pass == 1 || (ctx->primary_pass == -1 && mode == 1)) &&
                         2 * primary_need * sizeof(uint4) <= ctx->batch_budget;
    ka.primary = nullptr;
    if (primary) {
        const int pi = (int)(ctx->batches & 1u);
        const size_t need = primary_need;
        if (need > ctx->primary_cap) {
            RT_HIP(ctx, join_aux(ctx));
            RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            const size_t want = std::max<size_t>(
                need, std::min<size_t>(ctx->batch_budget / (2 * sizeof(uint4)), (size_t)owned_px * ctx->frame_batch));
            for (uint4*& b : ctx->d_primary) {
                if (b) RT_HIP(ctx, hipFree(b));
                b = nullptr;
            }
            ctx->primary_cap = 0;
            for (uint4*& b : ctx->d_primary) {
                const hipError_t ea = hipMalloc(reinterpret_cast<void**>(&b), want * 16);
                if (ea != hipSuccess) return fail(ctx, RT_E_NOMEM, std::string("primary records: ") + hipGetErrorString(ea));
            }
            ctx->primary_cap = want;
        }
        KernelArgs pka = ka;
        pka.primary = ctx->d_primary[pi];
        pka.queue_units = ctx->owned_tiles * frames;  // one unit per (frame, tile)
        pka.primary_tile_major = ctx->primary_tile_major ? 1u : 0u;
        const size_t image = mode == 2 ? mode2_bytes : mode1_bytes;
        // (the 64-VGPR variant is built at 256 threads only)
        const uint32_t min_waves = (mode == 2 || ctx->primary_threads != 256u) ? 0u : ctx->primary_min_waves;
        RT_HIP(ctx, rt_launch_primary(pka, mode, tris, image, mode == 2 ? 1024u : ctx->primary_threads, min_waves, S));
        ka.primary = pka.primary;
    }
    hipError_t e = rt_launch_pathtrace(ka, mode, tris, ctx->occ_threads, lds_bytes, blocks, S);
    ctx->last_blocks = blocks;
    ctx->last_passes = RT_PASS_PATH | (primary ? RT_PASS_PRIMARY : 0u) | (frame_par ? RT_PASS_RESOLVE : 0u);
    ctx->last_lds = (uint32_t)lds_bytes;
    if (e != hipSuccess) return hip_fail(ctx, "rt_pathtrace_kernel launch", e);
    if (frame_par) {
        // the accumulation is summed in frame order: after the previous batch's resolve
        if (ctx->batches > 0) RT_HIP(ctx, hipStreamWaitEvent(S, ctx->ev_resolved[(ctx->batches - 1) & 1u], 0));
        e = rt_launch_resolve(ctx->d_accum, ctx->d_out, ka.frame_light, ctx->width, ctx->height, ctx->tiles_x,
                              ctx->owned_tiles, ctx->rank, ctx->world, p.accumulation_index, p.compute_per_frame,
                              frames, ka.launch_clock ? ka.launch_clock + 2 : nullptr, S);
        if (e != hipSuccess) return hip_fail(ctx, "rt_resolve_frames_kernel launch", e);
        RT_HIP(ctx, hipEventRecord(ctx->ev_resolved[ctx->batches & 1u], S));
        ctx->batches += 1;
    }
    // every tile is claimed once and every wave makes one final failing claim
    ctx->queue_parity[si] ^= 1u;  // this launch zeroes the other half for the stream's next one
    if (si) {
        RT_HIP(ctx, hipEventRecord(ctx->ev_aux_done, S));
        ctx->aux_outstanding = true;
    }
    // A plain launch (not frame-parallel) reads and writes the accumulation and
    // the output on the primary stream; a later overlapped batch on the auxiliary
    // stream must follow it (its resolve writes both), not just the previous batch.
    if (!frame_par) ctx->primary_dirty = true;
    if (sched) ++ctx->sched_launches[si];
    return RT_OK;
}

// Queueing a frame is host bookkeeping only: the device is selected (a HIP call)
// only when the call launches the batch.
int rt_compute_frame(rt_ctx* ctx, uint32_t bounces) {
    if (!ctx || ctx->frame_batch <= 1) return rt_compute_frames(ctx, bounces, 1);
    if (ctx->pending_frames && bounces != ctx->pending_bounces) {
        RT_ENTER_NOFLUSH(ctx);
        const int rc = flush_frames(ctx);
        if (rc) return rc;
    }
    if (ctx->pending_frames == 0) {
        ctx->pending_bounces = bounces;
        if (ctx->params.accumulate) ctx->params.accumulation_index = ctx->k;  // src/renderer.rs:216-235
    }
    if (ctx->params.accumulate) ctx->k += 1;
    ctx->pending_frames += 1;
    if (ctx->pending_frames < ctx->frame_batch) return RT_OK;
    RT_ENTER_NOFLUSH(ctx);
    return flush_frames(ctx);
}

int rt_submit_frames(rt_ctx* ctx, uint32_t bounces, uint32_t count) {
    if (!ctx) return RT_E_INVALID;
    for (uint32_t i = 0; i < count; i++) {
        const int rc = rt_compute_frame(ctx, bounces);
        if (rc) return rc;
    }
    return RT_OK;
}

int rt_set_frame_batch(rt_ctx* ctx, uint32_t max_frames) {
    RT_ENTER(ctx);
    if (max_frames == 0 || max_frames > kMaxFrameBatch)
        return fail(ctx, RT_E_INVALID, "frame batch must be in [1, " + std::to_string(kMaxFrameBatch) + "]");
    ctx->frame_batch = max_frames;
    return RT_OK;
}

int rt_frame_batch(const rt_ctx* ctx, uint32_t* max_frames, uint32_t* pending) {
    if (!ctx || !max_frames || !pending) return RT_E_INVALID;
    *max_frames = ctx->frame_batch;
    *pending = ctx->pending_frames;
    return RT_OK;
}

int rt_flush(rt_ctx* ctx) {
    RT_ENTER(ctx);
    return RT_OK;
}

int rt_compute_frames(rt_ctx* ctx, uint32_t bounces, uint32_t frames) {
    RT_ENTER(ctx);
    if (frames == 0) return fail(ctx, RT_E_INVALID, "frames must be >= 1");
    if (ctx->params.accumulate) {  // src/renderer.rs:216-235 (`accumulate` is a bool there)
        ctx->params.accumulation_index = ctx->k;
        ctx->k += frames;
    }
    return dispatch_frames(ctx, bounces, frames);
}

int rt_synchronize(rt_ctx* ctx) {
    RT_ENTER(ctx);
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_copy_output_to_device(rt_ctx* ctx, void* dst_device, uint32_t bytes_per_row) {
    RT_ENTER(ctx);  // queued frames launched first: the copy sees the last frame's output
    if (!dst_device) return fail(ctx, RT_E_INVALID, "rt_copy_output_to_device: dst_device is NULL");
    if (ctx->world > 1)  // a rank's output holds only its own tiles: gather first (rt_gather_frame)
        return fail(ctx, RT_E_INVALID, "rt_copy_output_to_device: a rank context (world_size > 1) has no full frame");
    {
        hipPointerAttribute_t attr{};
        const hipError_t ea = hipPointerGetAttributes(&attr, dst_device);
        if (ea != hipSuccess || attr.type != hipMemoryTypeDevice || attr.device != ctx->device) {
            (void)hipGetLastError();
            return fail(ctx, RT_E_INVALID, "rt_copy_output_to_device: dst_device is not device memory of the context's device");
        }
    }
    if ((uint64_t)bytes_per_row < 4ull * ctx->width)
        return fail(ctx, RT_E_INVALID, "rt_copy_output_to_device: bytes_per_row < 4 * width");
    RT_HIP(ctx, hipMemcpy2DAsync(dst_device, bytes_per_row, ctx->d_out, 4u * (size_t)ctx->width,
                                 4u * (size_t)ctx->width, ctx->height, hipMemcpyDeviceToDevice, ctx->stream));
    return RT_OK;
}

int rt_read_output(rt_ctx* ctx, uint32_t* out) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_out, ctx->n_pixels * 4, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_read_output_pitched(rt_ctx* ctx, uint8_t* dst, uint32_t bytes_per_row) {
    RT_ENTER(ctx);
    if (!dst) return fail(ctx, RT_E_INVALID, "dst is NULL");
    if ((uint64_t)bytes_per_row < 4ull * ctx->width) return fail(ctx, RT_E_INVALID, "bytes_per_row < 4 * width");
    RT_HIP(ctx, hipMemcpy2DAsync(dst, bytes_per_row, ctx->d_out, 4ull * ctx->width, 4ull * ctx->width, ctx->height,
                                 hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

uint32_t rt_bytes_per_row(uint32_t width, uint32_t alignment) {
    if (alignment == 0 || (alignment & (alignment - 1)) != 0) return 0;
    const uint64_t v = 4ull * width;
    const uint64_t r = (v + alignment - 1) & ~(uint64_t)(alignment - 1);
    return r > 0xffffffffull ? 0u : (uint32_t)r;
}

// ---- device-side edit path (scene_edit.hip) --------------------------------

int rt_set_object_models(rt_ctx* ctx, const float* points, uint32_t triangle_count) {
    RT_ENTER(ctx);
    if (triangle_count && !points) return fail(ctx, RT_E_INVALID, "normalized_points is NULL");
    if (triangle_count > ctx->cap_tri) return fail(ctx, RT_E_CAPACITY, "more triangles than the buffer holds");
    int rc = sync_host_geometry(ctx);
    if (rc) return rc;
    // triangle -> object and sub-object -> object maps, per-object triangle ranges
    const uint32_t n_obj = (uint32_t)ctx->h_obj.size(), n_sub = (uint32_t)ctx->h_sub.size();
    std::vector<uint32_t> tri_obj(std::max<uint32_t>(triangle_count, 1), 0xffffffffu);
    std::vector<uint32_t> sub_obj(std::max<uint32_t>(n_sub, 1), 0xffffffffu);
    std::vector<uint2> obj_tris(std::max<uint32_t>(n_obj, 1), make_uint2(0, 0));
    for (uint32_t o = 0; o < n_obj; o++) {
        const rt_object_info& ob = ctx->h_obj[o];
        uint32_t first = 0, count = 0;
        for (uint32_t i = 0; i < ob.sub_object_count; i++) {
            const uint32_t si = ob.first_sub_object_index + i;
            const rt_sub_object_info& so = ctx->h_sub[si];
            if (count == 0) first = so.first_triangle_index;
            if (so.triangle_count && so.first_triangle_index != first + count)
                return fail(ctx, RT_E_INVALID, "object " + std::to_string(o) + ": sub-object triangles not contiguous");
            if ((uint64_t)so.first_triangle_index + so.triangle_count > triangle_count)
                return fail(ctx, RT_E_INVALID, "object " + std::to_string(o) + " has triangles without model points");
            sub_obj[si] = o;
            for (uint32_t t = 0; t < so.triangle_count; t++) tri_obj[so.first_triangle_index + t] = o;
            count += so.triangle_count;
        }
        obj_tris[o] = make_uint2(first, count);
    }
    auto alloc = [&](auto** p, size_t count) -> int {
        if (*p) return RT_OK;
        return dev_alloc(ctx, p, count);
    };
    if ((rc = alloc(&ctx->d_model, 9 * (size_t)ctx->n_tri_dev)) || (rc = alloc(&ctx->d_tri_object, ctx->n_tri_dev)) ||
        (rc = alloc(&ctx->d_sub_object, ctx->n_sub_dev)) || (rc = alloc(&ctx->d_object_tris, std::max(ctx->cap_obj, 1u))) ||
        (rc = alloc(&ctx->d_place, std::max(ctx->cap_obj, 1u))) ||
        (rc = upload_raw(ctx, ctx->d_model, points, (size_t)triangle_count * 36)) ||
        (rc = upload_raw(ctx, ctx->d_tri_object, tri_obj.data(), (size_t)triangle_count * 4)) ||
        (rc = upload_raw(ctx, ctx->d_sub_object, sub_obj.data(), (size_t)n_sub * 4)) ||
        (rc = upload_raw(ctx, ctx->d_object_tris, obj_tris.data(), (size_t)n_obj * 8)))
        return rc;
    ctx->model_tris = triangle_count;
    ctx->models_valid = true;
    return RT_OK;
}

int rt_update_objects(rt_ctx* ctx, const rt_object_transform* transforms, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !transforms) return fail(ctx, RT_E_INVALID, "transforms is NULL");
    if (count > ctx->h_obj.size()) return fail(ctx, RT_E_CAPACITY, "more transforms than objects");
    if (count == 0) return RT_OK;
    if (!ctx->d_model || !ctx->models_valid)
        return fail(ctx, RT_E_INVALID,
                    "object models missing or stale (object / sub-object ranges changed): call rt_set_object_models");
    void* p;
    int rc = staging(ctx, (size_t)count * sizeof(rt_scene::Placement), &p);
    if (rc) return rc;
    rt_scene::Placement* pl = static_cast<rt_scene::Placement*>(p);
    for (uint32_t o = 0; o < count; o++)
        rt_scene::placement(*reinterpret_cast<const rt_scene::ObjectTransform*>(&transforms[o]), pl[o]);
    if ((rc = staged_copy(ctx, ctx->d_place, (size_t)count * sizeof(rt_scene::Placement)))) return rc;
    RT_HIP(ctx, rt_launch_edit(ctx->d_model, ctx->d_tri_object, ctx->d_sub_object, ctx->d_object_tris, ctx->d_place,
                               count, ctx->model_tris, (uint32_t)ctx->h_sub.size(), ctx->d_tri, ctx->d_tri_bounds,
                               ctx->d_sub, ctx->d_obj, ctx->stream));
    ctx->geom_on_device = true;
    // the accelerator keeps its topology; its boxes (and the margin extent) follow the new bounds
    if (ctx->d_tri_bvh && ctx->tri_nodes && !ctx->tri_dirty) {
        RT_HIP(ctx, rt_launch_refit(ctx->d_tri_bvh, ctx->d_tri_prims, ctx->d_sub, ctx->d_tri_order,
                                    ctx->d_tri_level_off, ctx->tri_levels, ctx->d_tri_extent, ctx->stream));
        ctx->qnodes_dirty = true;
    }
    ctx->cones_dirty = true;  // the triangles changed
    ctx->ltris_dirty = true;
    return RT_OK;
}

int rt_read_triangles(rt_ctx* ctx, rt_scene_triangle* out, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !out) return fail(ctx, RT_E_INVALID, "out is NULL");
    if (count > ctx->cap_tri) return fail(ctx, RT_E_CAPACITY, "more triangles than the buffer holds");
    if (count == 0) return RT_OK;
    std::vector<RtTriangleHot> hot(count);
    std::vector<float4> b(2 * (size_t)count);
    RT_HIP(ctx, hipMemcpyAsync(hot.data(), ctx->d_tri, (size_t)count * sizeof(RtTriangleHot), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipMemcpyAsync(b.data(), ctx->d_tri_bounds, (size_t)count * 32, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    auto put = [](float* dst, const float4& v) {
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
    };
    for (uint32_t i = 0; i < count; i++) {
        rt_scene_triangle& t = out[i];
        std::memset(&t, 0, sizeof(t));
        unpack_triangle(hot[i], t.a, t.edge_ab, t.edge_ac, t.calc_normal, t.face_normal);
        put(t.min_bounds, b[2 * i]);
        put(t.max_bounds, b[2 * i + 1]);
    }
    return RT_OK;
}

int rt_read_object_info(rt_ctx* ctx, rt_object_info* out, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !out) return fail(ctx, RT_E_INVALID, "out is NULL");
    if (count > ctx->cap_obj) return fail(ctx, RT_E_CAPACITY, "more objects than the buffer holds");
    if (count == 0) return RT_OK;
    RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_obj, (size_t)count * 48, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_read_sub_object_info(rt_ctx* ctx, rt_sub_object_info* out, uint32_t count) {
    RT_ENTER(ctx);
    if (count && !out) return fail(ctx, RT_E_INVALID, "out is NULL");
    if (count > ctx->cap_sub) return fail(ctx, RT_E_CAPACITY, "more sub-objects than the buffer holds");
    if (count == 0) return RT_OK;
    RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_sub, (size_t)count * 32, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_read_accumulation(rt_ctx* ctx, float* out) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_accum, ctx->n_pixels * 16, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_ray_count(rt_ctx* ctx, uint64_t* out) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    unsigned long long v = 0;
    RT_HIP(ctx, hipMemcpyAsync(&v, ctx->d_counter, sizeof(v), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *out = v;
    return RT_OK;
}

int rt_set_brute_force(rt_ctx* ctx, int enable) {
    RT_ENTER(ctx);
    if (enable < 0 || enable > 2) return fail(ctx, RT_E_INVALID, "brute-force mode must be 0, 1 or 2");
    ctx->brute = enable;
    return RT_OK;
}

int rt_set_triangle_pruning(rt_ctx* ctx, int mode) {
    RT_ENTER(ctx);
    if (mode < 0 || mode > 2) return fail(ctx, RT_E_INVALID, "triangle pruning mode must be 0, 1 or 2");
    ctx->tri_prune_mode = mode;
    return RT_OK;
}

int rt_streamed_bytes(rt_ctx* ctx, uint64_t* out) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    unsigned long long v[2] = {0, 0};
    RT_HIP(ctx, hipMemcpyAsync(v, ctx->d_stream, sizeof(v), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *out = v[0];
    return RT_OK;
}

int rt_streamed_bytes_l2(rt_ctx* ctx, uint64_t* out) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    unsigned long long v[2] = {0, 0};
    RT_HIP(ctx, hipMemcpyAsync(v, ctx->d_stream, sizeof(v), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *out = v[1];
    return RT_OK;
}

// Exact variants of the schedule and the acceleration structures, for A/B measurements (the
// product reads no environment): every setting renders the same bits.
int rt_set_tuning(rt_ctx* ctx, const char* key, int32_t value) {
    RT_ENTER(ctx);
    if (!key) return fail(ctx, RT_E_INVALID, "rt_set_tuning: key is NULL");
    const std::string k(key);
    const int32_t v = value;
    auto range = [&](int32_t lo, int32_t hi) {
        return v >= lo && v <= hi ? RT_OK
                                  : fail(ctx, RT_E_INVALID, "rt_set_tuning: " + k + " must be in [" + std::to_string(lo) +
                                                                ", " + std::to_string(hi) + "]");
    };
    auto flag = [&](bool& field) {
        const int rc = range(0, 1);
        if (rc == RT_OK) field = v != 0;
        return rc;
    };
    int rc = RT_OK;
    if (k == "scene_in_lds") {
        if ((rc = range(0, 1)) == RT_OK) ctx->force_global_scene = v == 0;
    } else if (k == "lds_mode") {
        if ((rc = range(0, 2)) == RT_OK) ctx->max_lds_mode = v;
    } else if (k == "block_threads") {
        if (v != 0 && v != 256 && v != 512 && v != 1024)
            return fail(ctx, RT_E_INVALID, "rt_set_tuning: block_threads must be 0, 256, 512 or 1024");
        ctx->force_threads = (uint32_t)v;
        ctx->occ_blocks_per_cu = 0;
    } else if (k == "waves_per_cu") {
        if ((rc = range(0, 32)) == RT_OK) {
            ctx->waves_cap = (uint32_t)v;
            ctx->occ_blocks_per_cu = 0;
        }
    } else if (k == "tri_bvh") {
        if ((rc = flag(ctx->use_tri_bvh)) == RT_OK) ctx->tri_dirty = true;
    } else if (k == "tri_octants") {
        if ((rc = flag(ctx->use_tri_octants)) == RT_OK) ctx->tri_dirty = true;
    } else if (k == "tri_qnodes") {
        rc = flag(ctx->use_qnodes);
    } else if (k == "coop_leaves") {
        rc = flag(ctx->use_coop_leaves);
    } else if (k == "stage_subs") {
        rc = flag(ctx->stage_subs);
    } else if (k == "primary_pass") {
        if ((rc = range(-1, 1)) == RT_OK) ctx->primary_pass = v;
    } else if (k == "primary_threads") {
        if (v != 64 && v != 128 && v != 256 && v != 512 && v != 1024)
            return fail(ctx, RT_E_INVALID, "rt_set_tuning: primary_threads must be 64, 128, 256, 512 or 1024");
        ctx->primary_threads = (uint32_t)v;
    } else if (k == "primary_waves") {
        if (v != 0 && v != 8) return fail(ctx, RT_E_INVALID, "rt_set_tuning: primary_waves must be 0 or 8");
        ctx->primary_min_waves = (uint32_t)v;
    } else if (k == "primary_tile_major") {
        rc = flag(ctx->primary_tile_major);
    } else if (k == "sphere_bvh") {
        if ((rc = flag(ctx->use_bvh)) == RT_OK) ctx->slots_dirty = true;
    } else if (k == "sphere_leaf") {
        if ((rc = range(0, 64)) == RT_OK) {
            ctx->sphere_leaf_max = (uint32_t)v;
            ctx->slots_dirty = true;
        }
    } else if (k == "sphere_octants") {
        rc = flag(ctx->sphere_octants);
    } else if (k == "sphere_box_order") {
        if ((rc = flag(ctx->sphere_box_order)) == RT_OK) ctx->slots_dirty = true;
    } else if (k == "queue_stripes") {
        if ((rc = range(1, (int32_t)kQueueStripesMax)) == RT_OK) ctx->queue_stripes = (uint32_t)v;
    } else if (k == "trav_threshold") {
        if ((rc = range(0, 63)) == RT_OK) ctx->trav_threshold = (uint32_t)v;
    } else if (k == "drain_threshold") {
        if ((rc = range(0, 63)) == RT_OK) ctx->drain_threshold = (uint32_t)v;
    } else if (k == "drain_min_steps") {
        if ((rc = range(0, 1 << 20)) == RT_OK) ctx->drain_min_steps = (uint32_t)v;
    } else if (k == "leaf_batch") {
        if ((rc = range(0, 8)) == RT_OK) ctx->leaf_batch = (uint32_t)v;
    } else if (k == "tile_schedule") {
        if ((rc = range(0, 1)) == RT_OK) ctx->tile_schedule = (uint32_t)v;
    } else if (k == "frame_parallel") {
        rc = flag(ctx->frame_parallel);
    } else if (k == "batch_overlap") {
        rc = flag(ctx->batch_overlap);
    } else if (k == "batch_schedule") {
        rc = flag(ctx->batch_schedule);
    } else if (k == "unit_tile_major") {
        rc = flag(ctx->unit_tile_major);
    } else if (k == "batch_memory_mb") {
        if ((rc = range(1, 1 << 30)) == RT_OK) ctx->batch_budget = (size_t)v << 20;
    } else {
        return fail(ctx, RT_E_INVALID, "rt_set_tuning: unknown key " + k);
    }
    return rc;
}

int rt_set_tile_schedule(rt_ctx* ctx, uint32_t schedule) {
    RT_ENTER(ctx);
    if (schedule > 1) return fail(ctx, RT_E_INVALID, "tile schedule must be 0 (index order) or 1 (cost-ordered)");
    ctx->tile_schedule = schedule;
    for (int si = 0; si < 2; si++) {
        if (ctx->d_tile_sched[si])
            RT_HIP(ctx, hipMemsetAsync(ctx->d_tile_sched[si], 0, (4 * (size_t)ctx->owned_tiles + 2) * 4, ctx->stream));
        ctx->sched_launches[si] = 0;
    }
    return RT_OK;
}

int rt_tile_schedule_state(rt_ctx* ctx, uint32_t* order, uint32_t* costs) {
    RT_ENTER(ctx);
    // the primary stream's schedule: the one every single-frame launch and every
    // other overlapped batch follows
    const size_t n = ctx->owned_tiles;
    const uint32_t* st = ctx->d_tile_sched[0];
    const uint64_t launches = ctx->sched_launches[0];
    const bool on = ctx->tile_schedule && st;
    const uint32_t par = (uint32_t)(launches & 1u);  // the next launch's parity
    for (size_t i = 0; i < n && order; i++) order[i] = (uint32_t)i;
    if (order && on && launches)
        RT_HIP(ctx, hipMemcpyAsync(order, st + 2 * n + par * n, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (costs) {
        if (on && launches)  // what the last launch recorded
            RT_HIP(ctx, hipMemcpyAsync(costs, st + (par ^ 1u) * n, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        else
            std::memset(costs, 0, n * 4);
    }
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_reset_ray_count(rt_ctx* ctx) {
    RT_ENTER(ctx);
    RT_HIP(ctx, hipMemsetAsync(ctx->d_counter, 0, (1 + kDiagCounters) * sizeof(unsigned long long), ctx->stream));
    RT_HIP(ctx, hipMemsetAsync(ctx->d_stream, 0, 2 * sizeof(unsigned long long), ctx->stream));
    return RT_OK;
}

int rt_accumulation_index(const rt_ctx* ctx, uint32_t* out) {
    if (!ctx || !out) return RT_E_INVALID;
    *out = ctx->k;
    return RT_OK;
}

int rt_set_timing(rt_ctx* ctx, int enable) {
    RT_ENTER(ctx);
    ctx->timing = enable != 0;
    // The launch-clock slots are allocated (and zeroed) here rather than by the first timed
    // launch: callers switch timing on ahead of the region they time (bench.py), which then
    // holds no hipMalloc on its launch path.
    if (ctx->timing && !ctx->d_clock) {
        const int rc = dev_alloc(ctx, &ctx->d_clock, kClockWords * (size_t)kClockSlots);
        if (rc) return rc;
        RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return RT_OK;
}

int rt_last_dispatch_ms(rt_ctx* ctx, float* out_ms) {
    RT_ENTER(ctx);
    if (!out_ms) return fail(ctx, RT_E_INVALID, "out is NULL");
    int rc = collect_timing(ctx);
    if (rc) return rc;
    *out_ms = ctx->last_ms;
    return RT_OK;
}

int rt_dispatch_time_total(rt_ctx* ctx, double* total_ms, uint64_t* n_timed) {
    RT_ENTER(ctx);
    if (!total_ms || !n_timed) return fail(ctx, RT_E_INVALID, "out is NULL");
    int rc = collect_timing(ctx);
    if (rc) return rc;
    *total_ms = ctx->total_ms;
    *n_timed = ctx->n_timed;
    return RT_OK;
}

int rt_resolve_time_total(rt_ctx* ctx, double* total_ms, uint64_t* n_timed) {
    RT_ENTER(ctx);
    if (!total_ms || !n_timed) return fail(ctx, RT_E_INVALID, "out is NULL");
    int rc = collect_timing(ctx);
    if (rc) return rc;
    *total_ms = ctx->resolve_total_ms;
    *n_timed = ctx->n_resolve_timed;
    return RT_OK;
}

int rt_reset_timing(rt_ctx* ctx) {
    RT_ENTER(ctx);
    int rc = collect_timing(ctx);
    if (rc) return rc;
    ctx->total_ms = 0.0;
    ctx->n_timed = 0;
    ctx->resolve_total_ms = 0.0;
    ctx->n_resolve_timed = 0;
    ctx->last_ms = 0.0f;
    return RT_OK;
}

int rt_owned_pixel_count(const rt_ctx* ctx, uint32_t rank, uint32_t world_size, uint64_t* out) {
    if (!ctx || !out || world_size == 0 || rank >= world_size) return RT_E_INVALID;
    *out = (uint64_t)owned_tile_count(ctx->tiles_x * ctx->tiles_y, rank, world_size) * 64u;
    return RT_OK;
}

int rt_pack_owned_accumulation(rt_ctx* ctx, void* dst_device) {
    RT_ENTER(ctx);
    if (!dst_device) return fail(ctx, RT_E_INVALID, "dst is NULL");
    if (ctx->owned_tiles == 0) return RT_OK;
    hipError_t e = rt_launch_pack(ctx->d_accum, static_cast<float4*>(dst_device), ctx->width, ctx->height,
                                  ctx->tiles_x, ctx->owned_tiles, ctx->rank, ctx->world, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_pack_tiles_kernel launch", e);
    return RT_OK;
}

int rt_unpack_accumulation(rt_ctx* ctx, const void* src_device, uint32_t src_rank, uint32_t world_size,
                           uint32_t divisor) {
    RT_ENTER(ctx);
    if (!src_device || world_size == 0 || src_rank >= world_size || divisor == 0)
        return fail(ctx, RT_E_INVALID, "unpack: bad arguments");
    hipError_t e = rt_launch_unpack(static_cast<const float4*>(src_device), ctx->d_accum, ctx->d_out, ctx->width,
                                    ctx->height, ctx->tiles_x, ctx->tiles_x * ctx->tiles_y, src_rank, 1, world_size,
                                    0, 0xffffffffu, (float)divisor, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_unpack_tiles_kernel launch", e);
    return RT_OK;
}

int rt_unpack_accumulation_ranks(rt_ctx* ctx, const void* src_device, uint64_t stride_px, uint32_t world_size,
                                 uint32_t skip_rank, uint32_t divisor) {
    RT_ENTER(ctx);
    const uint64_t cap = (uint64_t)owned_tile_count(ctx->tiles_x * ctx->tiles_y, 0, world_size ? world_size : 1) * 64u;
    if (!src_device || world_size == 0 || divisor == 0 || stride_px < cap)
        return fail(ctx, RT_E_INVALID, "unpack: bad arguments (stride below the largest rank's block?)");
    hipError_t e = rt_launch_unpack(static_cast<const float4*>(src_device), ctx->d_accum, ctx->d_out, ctx->width,
                                    ctx->height, ctx->tiles_x, ctx->tiles_x * ctx->tiles_y, 0, world_size, world_size,
                                    stride_px, skip_rank, (float)divisor, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_unpack_tiles_kernel launch", e);
    return RT_OK;
}

int rt_pack_owned_output(rt_ctx* ctx, void* dst_device) {
    RT_ENTER(ctx);
    if (!dst_device) return fail(ctx, RT_E_INVALID, "dst is NULL");
    if (ctx->owned_tiles == 0) return RT_OK;
    hipError_t e = rt_launch_pack_output(ctx->d_out, static_cast<uint32_t*>(dst_device), ctx->width, ctx->height,
                                         ctx->tiles_x, ctx->tiles_x * ctx->tiles_y, ctx->rank, 1, ctx->world, 0,
                                         0xffffffffu, false, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_pack_output_kernel launch", e);
    return RT_OK;
}

int rt_unpack_output(rt_ctx* ctx, const void* src_device, uint32_t src_rank, uint32_t world_size) {
    RT_ENTER(ctx);
    if (!src_device || world_size == 0 || src_rank >= world_size) return fail(ctx, RT_E_INVALID, "unpack: bad arguments");
    hipError_t e = rt_launch_pack_output(ctx->d_out, const_cast<uint32_t*>(static_cast<const uint32_t*>(src_device)),
                                         ctx->width, ctx->height, ctx->tiles_x, ctx->tiles_x * ctx->tiles_y, src_rank, 1,
                                         world_size, 0, 0xffffffffu, true, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_pack_output_kernel launch", e);
    return RT_OK;
}

int rt_unpack_output_ranks(rt_ctx* ctx, const void* src_device, uint64_t stride_px, uint32_t world_size,
                           uint32_t skip_rank) {
    RT_ENTER(ctx);
    const uint64_t cap = (uint64_t)owned_tile_count(ctx->tiles_x * ctx->tiles_y, 0, world_size ? world_size : 1) * 64u;
    if (!src_device || world_size == 0 || stride_px < cap)
        return fail(ctx, RT_E_INVALID, "unpack: bad arguments (stride below the largest rank's block?)");
    hipError_t e = rt_launch_pack_output(ctx->d_out, const_cast<uint32_t*>(static_cast<const uint32_t*>(src_device)),
                                         ctx->width, ctx->height, ctx->tiles_x, ctx->tiles_x * ctx->tiles_y, 0,
                                         world_size, world_size, stride_px, skip_rank, true, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "rt_pack_output_kernel launch", e);
    return RT_OK;
}

int rt_debug_counters(rt_ctx* ctx, uint64_t* out, uint32_t n) {
    RT_ENTER(ctx);
    if (!out) return fail(ctx, RT_E_INVALID, "out is NULL");
    const size_t m = std::min<size_t>(n, kDiagCounters + kDiagWaveRecords);
    RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_counter + 1, m * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int rt_debug_check_leaf_certificates(rt_ctx* ctx, uint32_t* mismatches, uint32_t* valid, uint32_t* total) {
    RT_ENTER(ctx);
    if (!mismatches || !valid || !total) return fail(ctx, RT_E_INVALID, "NULL output");
    *mismatches = *valid = *total = 0;
    RT_HIP(ctx, join_aux(ctx));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t n = ctx->tri_prim_count;
    if (!ctx->d_tri_lcert || ctx->cones_dirty || n == 0 || ctx->tri_lcert_cap < (size_t)n * sizeof(TriLeafCert))
        return RT_OK;
    std::vector<TriLeafCert> dev(n);
    std::vector<SubObjectPrim> prims(n);
    std::vector<RtSubObject> subs(ctx->n_sub_dev);
    std::vector<RtTriangleHot> tris(ctx->n_tri_dev);
    RT_HIP(ctx, hipMemcpy(dev.data(), ctx->d_tri_lcert, n * sizeof(TriLeafCert), hipMemcpyDeviceToHost));
    RT_HIP(ctx, hipMemcpy(prims.data(), ctx->d_tri_prims, n * sizeof(SubObjectPrim), hipMemcpyDeviceToHost));
    RT_HIP(ctx, hipMemcpy(subs.data(), ctx->d_sub, subs.size() * sizeof(RtSubObject), hipMemcpyDeviceToHost));
    RT_HIP(ctx, hipMemcpy(tris.data(), ctx->d_tri, tris.size() * sizeof(RtTriangleHot), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; i++) {
        const RtSubObject& s = subs[std::min<uint32_t>(prims[i].sub, (uint32_t)subs.size() - 1u)];
        float lo[3], hi[3];
        for (int k = 0; k < 3; k++) {
            lo[k] = std::fmin(s.min_bounds[k], s.max_bounds[k]);
            hi[k] = std::fmax(s.min_bounds[k], s.max_bounds[k]);
        }
        const uint32_t n_tri = (uint32_t)tris.size();
        const uint32_t cnt = (s.triangle_count <= kLeafCertSlots && n_tri != 0u) ? s.triangle_count : 0u;
        float a[kLeafCertSlots][3], ab[kLeafCertSlots][3], ac[kLeafCertSlots][3], cn[kLeafCertSlots][3];
        for (uint32_t j = 0; j < cnt; ++j) {
            float fn[3];
            unpack_triangle(tris[std::min(s.first_triangle_index + j, n_tri - 1u)], a[j], ab[j], ac[j], cn[j], fn);
        }
        const TriLeafCert h = tricone::leafcert_build(cnt, a, ab, ac, cn, lo, hi);
        *mismatches += std::memcmp(&h, &dev[i], sizeof(h)) != 0;
        *valid += dev[i].w[7] != kLeafCertNone;
    }
    *total = n;
    return RT_OK;
}

int rt_launch_config(rt_ctx* ctx, uint32_t* threads, uint32_t* blocks, uint32_t* lds_bytes,
                     uint32_t* scene_in_lds) {
    RT_ENTER(ctx);  // the last launch: queued frames launched first
    if (!threads || !blocks || !lds_bytes || !scene_in_lds) return RT_E_INVALID;
    *threads = ctx->occ_threads;
    *blocks = ctx->last_blocks;
    *lds_bytes = ctx->last_lds;
    *scene_in_lds = ctx->occ_mode < 0 ? 0u : (uint32_t)ctx->occ_mode;
    return RT_OK;
}

int rt_last_launch_passes(rt_ctx* ctx, uint32_t* passes) {
    RT_ENTER(ctx);  // the last launch: queued frames launched first
    if (!passes) return RT_E_INVALID;
    *passes = ctx->last_passes;
    return RT_OK;
}

void* rt_stream(rt_ctx* ctx) {
    if (!ctx) return nullptr;
    // flush_frames may launch and allocate: on the context's device
    if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
    // work the caller orders on this stream follows every frame submitted so far
    if (flush_frames(ctx) != RT_OK || join_aux(ctx) != hipSuccess) return nullptr;
    ctx->primary_dirty = true;
    return (void*)ctx->stream;
}

}  // extern "C"

int rt_math_selftest(uint32_t which, uint64_t* mismatches, uint32_t* first_bad) {
    if (!mismatches || !first_bad || which > 6) return RT_E_INVALID;
    unsigned long long* d_bad = nullptr;
    uint32_t* d_first = nullptr;
    hipError_t e = hipMalloc(&d_bad, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc(&d_first, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(d_bad, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_first, 0xff, sizeof(uint32_t));
    if (e == hipSuccess) e = rt_launch_math_selftest(which, d_bad, d_first, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long bad = 0;
    if (e == hipSuccess) e = hipMemcpy(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(first_bad, d_first, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (d_bad) (void)hipFree(d_bad);
    if (d_first) (void)hipFree(d_first);
    if (e != hipSuccess) return RT_E_HIP;
    *mismatches = bad;
    return RT_OK;
}
