/*
 * rt_abi.h — C ABI of the MI355X path-tracing hot path.
 *
 * This is the drop-in boundary for juhotuho10/rust_GPU_raytracing's per-frame
 * compute path. In the reference, `Renderer` (src/renderer.rs) owns a
 * `DataBuffers` (src/buffers.rs) of 10 wgpu buffers + 2 textures and records
 * one compute pass of `compute_shader.wgsl::main` per frame. Here the same
 * surface is a handful of `extern "C"` functions over an opaque context that
 * owns hipMalloc'd buffers, a pinned staging ring and one HIP stream. The
 * Rust side would bind these with a plain `extern "C" { ... }` block (see
 * INTEGRATION.md); nothing in the signatures is a C++ or torch type.
 *
 * POD layouts below are byte-for-byte the reference's `#[repr(C)]` structs
 * (src/buffers.rs:7-129) — the host arrays the reference already builds can be
 * handed over with no conversion.
 *
 * Conventions
 *   - every call returns int: RT_OK (0) or a negative RT_E* code; the message
 *     of the last failure is available from rt_last_error(ctx).
 *   - host arrays passed in are copied before the call returns (async copies
 *     go through the context's pinned staging ring); the caller keeps
 *     ownership.
 *   - one context = one device + one stream; calls on one context are not
 *     thread-safe (the reference's Renderer is owned by the event-loop thread,
 *     src/main.rs:240-496).
 *   - all device work is stream-ordered, exactly like wgpu queue submission
 *     order (src/renderer.rs:249): an update issued before rt_compute_frame is
 *     visible to that frame's dispatch.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define RT_API __attribute__((visibility("default")))
#else
#define RT_API
#endif

#define RT_ABI_VERSION 12

/* ---- error codes ------------------------------------------------------- */
#define RT_OK 0
#define RT_E_INVALID -1   /* bad argument (null, size mismatch, index out of range) */
#define RT_E_HIP -2       /* HIP runtime call failed */
#define RT_E_NOMEM -3     /* host or device allocation failed */
#define RT_E_CAPACITY -4  /* update larger than the buffer created at rt_create (wgpu would panic) */
#define RT_E_NODEVICE -5  /* no HIP device / device index out of range */

/* ---- POD scene types: src/buffers.rs:7-129 ----------------------------- */

/* src/buffers.rs:9-22 (Params) / compute_shader.wgsl:43-58. 48 bytes. */
typedef struct rt_params {
    uint32_t screen_width;
    uint32_t accumulation_index;
    uint32_t accumulate;
    uint32_t sphere_count;
    uint32_t object_count;
    uint32_t compute_per_frame;
    uint32_t texture_width;
    uint32_t texture_height;
    uint32_t texture_count; /* `textue_count` in the reference */
    uint32_t env_map_width;
    uint32_t env_map_height;
    uint32_t _padding;
} rt_params;

/* src/buffers.rs:26-29 (RayCamera). 16 bytes. */
typedef struct rt_ray_camera {
    float origin[3];
    uint32_t _padding;
} rt_ray_camera;

/* src/buffers.rs:33-36 (Ray): a cached per-pixel camera ray direction. 16 bytes. */
typedef struct rt_ray {
    float direction[3];
    uint32_t _padding;
} rt_ray;

/* src/buffers.rs:40-45 (SceneSphere). 32 bytes. */
typedef struct rt_scene_sphere {
    float position[3];
    float radius;
    uint32_t material_index;
    uint32_t _padding[3];
} rt_scene_sphere;

/* src/buffers.rs:49-64 (SceneTriangle), built by SceneTriangle::new
 * (src/buffers.rs:66-95): edge_ab = b-a, edge_ac = c-a,
 * calc_normal = edge_ab x edge_ac, face_normal = normalize(calc_normal).
 * 112 bytes. min/max_bounds are host-only (the kernel never reads them). */
typedef struct rt_scene_triangle {
    float a[3];           uint32_t _padding0;
    float edge_ab[3];     uint32_t _padding1;
    float edge_ac[3];     uint32_t _padding2;
    float calc_normal[3]; uint32_t _padding3;
    float face_normal[3]; uint32_t _padding4;
    float min_bounds[3];  uint32_t _padding5;
    float max_bounds[3];  uint32_t _padding6;
} rt_scene_triangle;

/* src/buffers.rs:100-109 (SceneMaterial). 32 bytes. */
typedef struct rt_scene_material {
    uint32_t texture_index;
    float roughness;
    float emission_power;
    float specular;
    float specular_scatter;
    float glass;
    float refraction_index;
    uint32_t _padding;
} rt_scene_material;

/* src/buffers.rs:113-120 (ObjectInfo). 48 bytes. */
typedef struct rt_object_info {
    float min_bounds[3];
    uint32_t first_sub_object_index;
    float max_bounds[3];
    uint32_t sub_object_count;
    uint32_t material_index;
    uint32_t _padding[3];
} rt_object_info;

/* src/buffers.rs:124-129 (SubObjectInfo). 32 bytes. */
typedef struct rt_sub_object_info {
    float min_bounds[3];
    uint32_t first_triangle_index;
    float max_bounds[3];
    uint32_t triangle_count;
} rt_sub_object_info;

/* ---- context ------------------------------------------------------------ */

typedef struct rt_ctx rt_ctx;

/* Everything DataBuffers::new (src/buffers.rs:159-170) receives, plus the
 * framebuffer height (Params carries only the width) and the device.
 * Array capacities are fixed here, as wgpu buffer sizes are fixed at
 * creation; later rt_update_* calls must fit. Zero-length arrays are allowed
 * (the reference needs a dummy element because WGSL arrays cannot be empty). */
typedef struct rt_create_info {
    uint32_t width;
    uint32_t height;
    int32_t device;              /* HIP device ordinal */
    uint32_t _reserved;
    rt_ray_camera camera;        /* binding 3 */
    const rt_ray* camera_rays;   /* binding 1, width*height entries */
    const rt_scene_material* materials; uint32_t material_count;   /* binding 4 */
    const rt_scene_sphere* spheres;     uint32_t sphere_count;     /* binding 5 */
    const rt_scene_triangle* triangles; uint32_t triangle_count;   /* binding 7 */
    const rt_object_info* objects;      uint32_t object_count;     /* binding 8 */
    const rt_sub_object_info* sub_objects; uint32_t sub_object_count; /* binding 10 */
    rt_params params;            /* binding 0: initial Params (Renderer::new, src/main.rs:131-144) */
    /* Tile partition for multi-GPU: the image is cut into 8x8
     * pixel tiles, tile t is rendered by rank (t % world_size). A context
     * with world_size == 1 renders every pixel, as the reference does. */
    uint32_t rank;
    uint32_t world_size;
} rt_create_info;

/* Renderer::new -> DataBuffers::new (src/renderer.rs:42-101,
 * src/buffers.rs:159-298). Allocates and fills every device buffer. Unlike the
 * reference (accumulation created uninitialised, src/buffers.rs:217-222) the
 * accumulation buffer starts zeroed. The renderer's accumulation counter k
 * starts at 1 (src/renderer.rs:96). */
RT_API int rt_create(const rt_create_info* info, rt_ctx** out_ctx);
RT_API void rt_destroy(rt_ctx* ctx);
RT_API const char* rt_last_error(const rt_ctx* ctx); /* never NULL; "" when no error */
RT_API int rt_abi_version(void);
/* Identity of this build: the hash of the sources, headers and compiler flags it
 * was compiled from (rust_gpu_raytracing_amd/build.py: source_hash). */
RT_API const char* rt_build_hash(void);

/* DataBuffers::update_texture_buffer (src/buffers.rs:479-511): `layers`
 * RGBA8 (sRGB-encoded, Rgba8UnormSrgb) images of width x height, tightly
 * packed, row 0 first. Resizes the texture array when the size changes. */
RT_API int rt_upload_textures(rt_ctx* ctx, const uint8_t* rgba8, uint32_t width, uint32_t height, uint32_t layers);
/* DataBuffers::update_environment_map_buffer (src/buffers.rs:513-539). */
RT_API int rt_upload_env_map(rt_ctx* ctx, const uint8_t* rgba8, uint32_t width, uint32_t height);

/* DataBuffers::update_accumulation (src/buffers.rs:557-559): write Params. */
RT_API int rt_update_params(rt_ctx* ctx, const rt_params* params);
/* DataBuffers::reset_accumulation (src/buffers.rs:545-555): zero the
 * accumulation buffer and write Params; also resets the context's
 * accumulation counter to params->accumulation_index (Renderer sets it to 1,
 * src/renderer.rs:131-151). */
RT_API int rt_reset_accumulation(rt_ctx* ctx, const rt_params* params);

/* DataBuffers::update_* (src/buffers.rs:541-595) and the camera write in
 * Renderer::on_update (src/renderer.rs:116-125). Writes start at element 0;
 * `count` must not exceed the capacity given at rt_create. */
RT_API int rt_update_ray_directions(rt_ctx* ctx, const rt_ray* rays, uint32_t count);
RT_API int rt_update_camera(rt_ctx* ctx, const rt_ray_camera* camera);

/* Device-side primary rays: instead of reading camera_rays,
 * the kernel computes each pixel's direction with the per-pixel arithmetic of
 * Camera::recalculate_ray_directions (src/camera.rs:139-182) from the camera's
 * inverse projection and inverse view (column-major 4x4 f32, glam layout), in
 * f32 with glam's operation order -- the same bits the host generator would
 * upload. Stays in effect until the next rt_update_ray_directions. */
RT_API int rt_update_camera_matrices(rt_ctx* ctx, const float inverse_projection[16], const float inverse_view[16]);
RT_API int rt_update_spheres(rt_ctx* ctx, const rt_scene_sphere* spheres, uint32_t count);
RT_API int rt_update_triangles(rt_ctx* ctx, const rt_scene_triangle* triangles, uint32_t count);
RT_API int rt_update_object_info(rt_ctx* ctx, const rt_object_info* objects, uint32_t count);
RT_API int rt_update_sub_object_info(rt_ctx* ctx, const rt_sub_object_info* sub_objects, uint32_t count);
RT_API int rt_update_materials(rt_ctx* ctx, const rt_scene_material* materials, uint32_t count);

/* The compute pass of Renderer::compute_frame (src/renderer.rs:238-249):
 * one launch of the path-tracing kernel with the Params currently on the
 * device. `bounces` is the per-path bounce limit (the reference hard-codes
 * 10, compute_shader.wgsl:150). Asynchronous. */
RT_API int rt_dispatch(rt_ctx* ctx, uint32_t bounces);

/* Renderer::compute_frame (src/renderer.rs:201-252): if Params.accumulate
 * is 1, write Params with accumulation_index = k and then k += 1; then
 * rt_dispatch. Asynchronous. With frame batching (below) the frame may only be
 * queued: an error of its launch (a failed allocation or launch) is then returned
 * by the call that launches the batch -- the rt_compute_frame that fills it, or
 * the next other entry point on the context. */
RT_API int rt_compute_frame(rt_ctx* ctx, uint32_t bounces);

/* `frames` consecutive rt_compute_frame calls fused into one launch: each
 * pixel runs its frames back to back on one lane, so the accumulation, the
 * packed output and the ray count afterwards are exactly those of the
 * sequence of calls (the per-frame outputs in between are never observable:
 * the reference only reads output_data after a frame, src/renderer.rs:254).
 * Used by the multi-GPU bench, where each rank advances its tiles by N frames
 * per step. frames >= 1. A batch whose per-frame buffers (32 B per owned pixel,
 * frame and sample) would exceed the batch budget -- an eighth of the device's
 * memory, tuning "batch_memory_mb" -- runs as consecutive launches of as many
 * frames as fit, with the same results. Asynchronous. */
RT_API int rt_compute_frames(rt_ctx* ctx, uint32_t bounces, uint32_t frames);

/* `count` consecutive rt_compute_frame calls made in one call (new, ABI 10): the loop a
 * native host runs around rt_compute_frame, for callers whose per-call overhead is not
 * negligible (the Python mirror: ~2 us per ctypes call, 40 us per 20-frame bench step at
 * N GPUs, where a rank's launch is 0.7 ms). Frame batching applies exactly as to the single
 * calls; results are identical. Stops at the first failing call. Asynchronous. */
RT_API int rt_submit_frames(rt_ctx* ctx, uint32_t bounces, uint32_t count);

/* Frame batching (new; the reference submits one dispatch per compute_frame,
 * src/renderer.rs:238-249, and wgpu runs it later, asynchronously). With
 * max_frames > 1, rt_compute_frame queues its frame (Params and k advance as
 * always) and one launch renders the queued frames once max_frames are queued,
 * when the bounce count changes, or before ANY other call on the context
 * (readback, update, sync, timing, destroy). Every frame is traced in full.
 * Accumulating batches are frame-parallel: each (frame, 8x8 tile) is a unit of
 * the launch's work queue, each path's light goes to a per-(frame, sample)
 * buffer, and a resolve pass adds them to the accumulation in the reference's
 * order (frame k's samples, then frame k+1's: compute_shader.wgsl:156-164), so
 * the accumulation, the packed output, the ray count and k after the batch are
 * bit-identical to the single-frame dispatches'; what changes is that the
 * persistent grid's fill and drain are paid once per batch, and that a tile
 * split over N GPUs keeps N x the units per launch. Non-accumulating batches
 * (every frame the same frame) run each pixel's frames back to back on a lane.
 * The default is RT_DEFAULT_FRAME_BATCH (ABI 11; it was 1, one launch per frame): a
 * host that mirrors the reference's event loop -- one rt_compute_frame per frame and
 * a display copy every few frames (src/renderer.rs:201-283, src/main.rs:88-92,
 * 365-375) -- gets launches of the frames between two displays without calling
 * this. 1 launches each frame at once.
 * max_frames in [1, 64]. rt_frame_batch reports the setting and the frames
 * queued; rt_flush launches them now. */
#define RT_DEFAULT_FRAME_BATCH 16
RT_API int rt_set_frame_batch(rt_ctx* ctx, uint32_t max_frames);
RT_API int rt_frame_batch(const rt_ctx* ctx, uint32_t* max_frames, uint32_t* pending);
RT_API int rt_flush(rt_ctx* ctx);

/* Blocks until all work on the context's stream has finished. */
RT_API int rt_synchronize(rt_ctx* ctx);

/* Readback (new: the reference only blits output_data to the swapchain,
 * src/renderer.rs:254-283). Synchronous; whole framebuffer, row-major
 * width*height. Pixels of tiles owned by another rank are left as they were
 * (zero unless written). */
RT_API int rt_read_output(rt_ctx* ctx, uint32_t* rgba8_out);
RT_API int rt_read_accumulation(rt_ctx* ctx, float* rgba_f32_out);

/* Display readback (Renderer::update_texture + calculate_bytes_per_row,
 * src/renderer.rs:254-295): the packed RGBA8 output (byte order R, G, B, A:
 * the Rgba8Unorm texel the reference copies into its display texture) written
 * row by row into `dst`, each row `bytes_per_row` bytes apart (>= 4*width; the
 * reference's wgpu copy needs a multiple of 256, which is what forces its
 * window width to a multiple of 64 pixels, src/main.rs:51-53 -- any pitch
 * works here). Padding bytes are left untouched. Synchronous. */
RT_API int rt_read_output_pitched(rt_ctx* ctx, uint8_t* dst, uint32_t bytes_per_row);

/* Renderer::update_texture on the device (new, ABI 11): the copy_buffer_to_texture of
 * src/renderer.rs:254-283 -- the packed RGBA8 output copied row by row into device
 * memory at `dst_device` (a display texture's staging buffer on the context's device),
 * rows `bytes_per_row` bytes apart (>= 4*width; padding untouched). Stream-ordered
 * after the frames submitted so far (queued frames are launched first), asynchronous:
 * the display observation point of a render loop, with no PCIe transfer and no host
 * wait, as in the reference (which never reads the frame back to the host).
 * RT_E_INVALID (ABI 12) when `dst_device` is not device memory of the context's device,
 * or on a rank context (world_size > 1), whose output holds only its own tiles. */
RT_API int rt_copy_output_to_device(rt_ctx* ctx, void* dst_device, uint32_t bytes_per_row);

/* calculate_bytes_per_row (src/renderer.rs:285-295): 4*width rounded up to
 * `alignment` (a power of two; the reference uses wgpu's 256). 0 on bad input. */
RT_API uint32_t rt_bytes_per_row(uint32_t width, uint32_t alignment);

/* Counted ray segments (every trace_ray call: primary + bounce, a path that
 * escapes to the environment stops counting), summed over all dispatches
 * since creation or the last rt_reset_ray_count. Synchronous. */
RT_API int rt_ray_count(rt_ctx* ctx, uint64_t* out);
RT_API int rt_reset_ray_count(rt_ctx* ctx);

/* Brute-force mode (BASELINE.json config 5, "brute-force LDS-tiled intersect
 * stress"): with enable = 1 later launches run the reference's own sweeps --
 * every sphere (check_spheres, compute_shader.wgsl:355-404), every object's and
 * sub-object's box and the triangles of those hit (check_triangles, :422-517) --
 * with no acceleration structure: a wavefront over the live paths, each
 * workgroup streaming the sub-object records through LDS in tiles and testing
 * them with broadcast reads. enable = 2 (ABI 11): the same sweeps with the
 * records streamed through the scalar cache by each wave (no LDS tile; a scene
 * without triangles has none to stream and runs mode 1's kernel: rt_last_launch_passes
 * says which ran). Same results, bit for bit, as the accelerated default (0); other
 * values are RT_E_INVALID. The scene's spheres, materials and objects must fit in LDS.
 * rt_streamed_bytes: the tile-streaming term of SURVEY §8d for those launches --
 * 32 B x the swept sub-objects per started 256 rays of each bounce level, its fixed
 * convention -- since creation or the last rt_reset_ray_count. rt_streamed_bytes_l2
 * (ABI 12): the sub-object bytes the sweeps actually read from L2 (per LDS tile and
 * workgroup in mode 1, per wave in mode 2). Synchronous. */
RT_API int rt_set_brute_force(rt_ctx* ctx, int enable);
RT_API int rt_streamed_bytes(rt_ctx* ctx, uint64_t* out);
RT_API int rt_streamed_bytes_l2(rt_ctx* ctx, uint64_t* out);

/* Distance pruning of the triangle walk (new; ABI 8, modes since ABI 9). The
 * reference sweeps every object -> sub-object -> triangle
 * (compute_shader.wgsl:422-517); the accelerator replaces the sweep by a walk that
 * culls boxes the ray misses, which is exact by construction.
 * mode 1 (the default): certified pruning -- once a triangle is hit at t, a triangle
 * of a leaf entered beyond t is also skipped (not loaded) when the leaf box, inflated
 * by a derived bound on the f32 error of the reference's triangle test for that
 * triangle (its own normal and two coefficients, the leaf's certificate, tri_cone.h;
 * ABI 10), is entered beyond t; exact by construction. Walks of an
 * LDS-resident accelerator use box culling in this mode. 0: box culling only. 2: the relative slack of
 * ABI 8 (skip boxes entered beyond t * (1 + 1/64) + 2^-10 (|o| + extent) / |d|):
 * faster on scenes without coherent normals, NOT exact -- rays nearly in a
 * triangle's plane near their origin can get another triangle than the sweep's
 * (tests/test_tri_accel_cpu.py builds such rays). Walks of the octant-ordered
 * layouts visit near boxes first in every mode. This call is the only way to select
 * mode 2 (the library reads no environment). Synchronous. */
RT_API int rt_set_triangle_pruning(rt_ctx* ctx, int mode);

/* Exact variants of the launch schedule and of the acceleration structures (new, ABI 12;
 * they were environment variables read at rt_create up to ABI 11), for A/B measurements:
 * every setting renders the same bits as the default. Takes effect from the next launch.
 * Keys and values (default first):
 *   "scene_in_lds" 1|0, "lds_mode" 2|1|0 (highest LDS staging mode), "block_threads"
 *   0|256|512|1024 (0: by occupancy), "waves_per_cu" 0..32 (0: 16), "trav_threshold" 0..63
 *   (0: by scene), "drain_threshold" 0..63 (32), "drain_min_steps" (64), "leaf_batch" 0..8
 *   (0: by scene), "queue_stripes" 1..64 (32), "tile_schedule" 1|0, "frame_parallel" 1|0,
 *   "batch_overlap" 1|0, "batch_schedule" 0|1, "unit_tile_major" 1|0, "batch_memory_mb"
 *   (an eighth of device memory), "sphere_bvh" 1|0, "sphere_leaf" 0..64 (0: default),
 *   "sphere_octants" 1|0, "sphere_box_order" 1|0, "tri_bvh" 1|0 (0: the reference's sweep),
 *   "tri_octants" 1|0, "tri_qnodes" 1|0, "coop_leaves" 1|0, "stage_subs" 1|0,
 *   "primary_pass" -1|0|1 (-1: by scene), "primary_threads" 256|64|128|512|1024,
 *   "primary_waves" 8|0, "primary_tile_major" 1|0.
 * RT_E_INVALID for an unknown key or a value out of range. */
RT_API int rt_set_tuning(rt_ctx* ctx, const char* key, int32_t value);

/* Tile claim order (new; the reference dispatches a plain grid,
 * src/renderer.rs:238-249). 0 = tile index order. 1 = cost-ordered (the
 * default): every launch records the rays each of its tiles took, and the
 * first workgroup of a launch to run out of tiles sorts the previous launch's
 * costs (most rays first) into the claim order of the next launch, while the
 * rest of the grid drains its last paths. Launches then end on cheap tiles
 * rather than on long paths. Active for launches in which every wave takes
 * at least 4 tiles on average (else the order cannot matter and the sort
 * would lengthen a short launch). Pixels are independent, so the image is
 * bit-identical under any order. Setting a schedule discards recorded costs
 * and orders (the next two launches run in index order). Asynchronous. */
RT_API int rt_set_tile_schedule(rt_ctx* ctx, uint32_t schedule);
/* The claim order the next launch uses (order[q] = local tile claimed at
 * queue position q; the identity when none is sorted yet) and the rays per
 * tile recorded by the last launch (zero once a later launch sorted them).
 * Either pointer may be NULL; each holds the rank's owned tile count
 * (rt_owned_pixel_count / 64). Synchronous. */
RT_API int rt_tile_schedule_state(rt_ctx* ctx, uint32_t* order, uint32_t* costs);

/* Current accumulation counter k (the value the next rt_compute_frame uses). */
RT_API int rt_accumulation_index(const rt_ctx* ctx, uint32_t* out);

/* Timing of path-tracing launches, enabled by rt_set_timing(ctx, 1) before them:
 * each timed launch's span on the device clock, from the start of its first
 * workgroup to the end of its last (s_memrealtime, the same interval rocprofv3's
 * kernel trace reports; overlapped batches' spans overlap). rt_last_dispatch_ms:
 * the last one (milliseconds). Synchronous. */
RT_API int rt_set_timing(rt_ctx* ctx, int enable);
RT_API int rt_last_dispatch_ms(rt_ctx* ctx, float* out_ms);
/* Sum of the timed launch spans since the last rt_reset_timing, and how many
 * launches were timed (read back in bulk on this call, so timing a long run adds
 * no host sync per frame). */
RT_API int rt_dispatch_time_total(rt_ctx* ctx, double* total_ms, uint64_t* n_timed);
/* The same for the resolve pass of timed frame-parallel batches
 * (rt_resolve_frames_kernel: each pixel's lights added to its accumulation in
 * frame order, the last frame's RGBA8 packed), which the path kernel's span above
 * does not include. n_timed counts the batches that had one. */
RT_API int rt_resolve_time_total(rt_ctx* ctx, double* total_ms, uint64_t* n_timed);
RT_API int rt_reset_timing(rt_ctx* ctx);

/* Multi-GPU gather support. The pixels owned by this context's
 * rank, in tile order, are packed into / unpacked from a contiguous device
 * buffer so one RCCL collective moves them. Sizes are in pixels. */
RT_API int rt_owned_pixel_count(const rt_ctx* ctx, uint32_t rank, uint32_t world_size, uint64_t* out);
/* Pack this rank's accumulation (float4 per pixel) into device memory `dst`
 * (rt_owned_pixel_count * 16 bytes). Stream-ordered on the context's stream. */
RT_API int rt_pack_owned_accumulation(rt_ctx* ctx, void* dst_device);
/* Unpack a block packed by `src_rank` of `world_size` into this context's
 * accumulation buffer and re-pack the RGBA8 output for those pixels with
 * the given accumulation divisor (k*c, src/compute_shader.wgsl:166). */
RT_API int rt_unpack_accumulation(rt_ctx* ctx, const void* src_device, uint32_t src_rank, uint32_t world_size,
                           uint32_t divisor);
/* The same for the packed RGBA8 output (one u32 per pixel, rt_owned_pixel_count
 * * 4 bytes), copied as is: the gather of a non-accumulating render
 * (Params.accumulate == 0 never writes the accumulation, compute_shader.wgsl:171-178). */
RT_API int rt_pack_owned_output(rt_ctx* ctx, void* dst_device);
RT_API int rt_unpack_output(rt_ctx* ctx, const void* src_device, uint32_t src_rank, uint32_t world_size);
/* One launch for a whole gather: `src_device` holds world_size consecutive
 * blocks of `stride_px` pixels (>= rank 0's rt_owned_pixel_count, the largest),
 * block r packed by rank r; every block except skip_rank's (the destination's
 * own tiles, already in place; pass world_size or more to unpack all) is
 * unpacked as rt_unpack_accumulation / rt_unpack_output would. */
RT_API int rt_unpack_accumulation_ranks(rt_ctx* ctx, const void* src_device, uint64_t stride_px,
                                        uint32_t world_size, uint32_t skip_rank, uint32_t divisor);
RT_API int rt_unpack_output_ranks(rt_ctx* ctx, const void* src_device, uint64_t stride_px, uint32_t world_size,
                                  uint32_t skip_rank);

/* Launch geometry of the last rt_dispatch (diagnostics): workgroup size in
 * threads, workgroups launched, dynamic LDS bytes per workgroup, and the LDS
 * staging mode (0: scene in global memory, 1: spheres/materials/objects/sphere
 * BVH staged in LDS, 2: also the triangle accelerator). */
RT_API int rt_launch_config(rt_ctx* ctx, uint32_t* threads, uint32_t* blocks, uint32_t* lds_bytes,
                            uint32_t* scene_in_lds);

/* The kernels the last rt_dispatch ran (diagnostics, ABI 7), a mask of RT_PASS_*:
 * the path kernel, the coherent primary-ray pre-pass, the batch resolve pass, or the
 * brute-force sweep kernel instead of the path kernel (with RT_PASS_BRUTE_STREAM, ABI 12:
 * its scalar-cache variant, rt_set_brute_force mode 2). Bit 32 (RT_PASS_TREELET, an ABI-12
 * treelet wavefront measured 2.9x slower than the path kernel on C5 and removed) is not set. */
#define RT_PASS_PATH 1u
#define RT_PASS_PRIMARY 2u
#define RT_PASS_RESOLVE 4u
#define RT_PASS_BRUTE 8u
#define RT_PASS_BRUTE_STREAM 16u
RT_API int rt_last_launch_passes(rt_ctx* ctx, uint32_t* passes);

/* Diagnostic counters (filled only by builds compiled with -DRT_DIAG or
 * -DRT_DIAG_TAIL, zeros otherwise): out[0..n) receives up to 8 u64 counters
 * (tools/diag_split.py, tools/tail_probe.py), then, for n > 8, per-wave
 * (start, end) real-time stamps of the last launch (-DRT_DIAG_TAIL). */
RT_API int rt_debug_counters(rt_ctx* ctx, uint64_t* out, uint32_t n);

/* Diagnostics (ABI 10): re-derives every leaf certificate of the certified triangle walk
 * (tri_cone.h) on the host from the device's current leaf records,
 * sub-objects and triangles, and compares them with the records the device built.
 * *mismatches = differing records, *valid = records that carry a certificate, *total =
 * leaf records (all 0 when the last launch read no certificates). */
RT_API int rt_debug_check_leaf_certificates(rt_ctx* ctx, uint32_t* mismatches, uint32_t* valid, uint32_t* total);

/* Device self-check of the kernel's fast exact-arithmetic helpers against the
 * IEEE operations they replace, over every f32 input (current device):
 * which 0 = sqrt on {+-0} U [2^-96, inf], 1..4 = x / 2pi, x / pi, x / 255,
 * x / 10; 5: the Box-Muller log, 6: its cos, on every value random01 returns.
 * *mismatches = number of differing results (0 = bit-exact),
 * *first_bad = smallest differing input's bit pattern (0xffffffff if none). */
RT_API int rt_math_selftest(uint32_t which, uint64_t* mismatches, uint32_t* first_bad);

/* The context's HIP stream (hipStream_t), for callers that want to order
 * their own device work (e.g. an RCCL collective) after a frame. */
RT_API void* rt_stream(rt_ctx* ctx);

/* The 256-entry sRGB -> linear table the kernel decodes Rgba8UnormSrgb
 * texels with (IEC 61966-2-1, rounded to f32). For tests. */
RT_API int rt_srgb_table(float out[256]);

/* ---- several GPUs in one process (SURVEY §5, §8b threading row, §8e) -----
 *
 * The reference renders on one adapter (src/main.rs:636-665). A group is N
 * contexts in this process -- rank r on devices[r], world N: 8x8 tile t is
 * rendered by rank t % N, with global pixel indices for the RNG seeds, so the
 * assembled frame is bit-identical to one GPU's -- each driven by its own host
 * thread, plus one RCCL communicator per device (ncclCommInitAll; librccl is
 * loaded on the first rt_create_multi). Rendering needs no communication;
 * rt_gather_frame assembles the frame on a root device over xGMI.
 *
 * `info` describes the whole frame and scene exactly as for rt_create (rank 0,
 * world_size 0 or 1; its `device` is ignored). Host arrays passed to group calls
 * are copied by every device before the call returns. Calls on one group are not
 * thread-safe. rt_group_compute_frame is asynchronous (each device's thread
 * queues or launches its share); a failure there is returned by the next
 * synchronous group call. rt_group_context gives rank r's context for the
 * single-context entry points -- only while the group is idle (after
 * rt_group_synchronize or a synchronous group call).
 * Group errors: rt_group_last_error(g) (rt_last_error(NULL) for rt_create_multi). */
typedef struct rt_group rt_group;

RT_API int rt_create_multi(const rt_create_info* info, const int32_t* devices, uint32_t n_devices, rt_group** out);
/* rt_create_multi with flags (new, ABI 11). RT_GROUP_COPY_TRANSPORT: no RCCL
 * communicators; rt_gather_frame moves each rank's packed block to the root with a
 * stream-ordered device-to-device copy (hipMemcpyPeerAsync on the sender's stream,
 * after the root's previous unpack; the root's unpack waits for every copy), and a
 * device may be listed more than once -- several ranks of one group on one GPU, which
 * runs the group's N-rank logic (one host thread and context per rank, tile ownership,
 * the root's N receive slots) on a one-GPU machine, or a group where RCCL is absent.
 * The assembled frame is the same bits either way. flags 0 == rt_create_multi. */
#define RT_GROUP_COPY_TRANSPORT 1u
RT_API int rt_create_multi_ex(const rt_create_info* info, const int32_t* devices, uint32_t n_devices, uint32_t flags,
                              rt_group** out);
RT_API void rt_destroy_multi(rt_group* g);
RT_API const char* rt_group_last_error(const rt_group* g);
RT_API uint32_t rt_group_size(const rt_group* g);
RT_API rt_ctx* rt_group_context(rt_group* g, uint32_t rank);

/* Renderer::compute_frame (src/renderer.rs:201-252) on every device's share. */
RT_API int rt_group_compute_frame(rt_group* g, uint32_t bounces);
RT_API int rt_group_set_frame_batch(rt_group* g, uint32_t max_frames);
RT_API int rt_group_flush(rt_group* g);
RT_API int rt_group_synchronize(rt_group* g);
RT_API int rt_group_update_params(rt_group* g, const rt_params* params);
RT_API int rt_group_reset_accumulation(rt_group* g, const rt_params* params);
RT_API int rt_group_update_camera(rt_group* g, const rt_ray_camera* camera);
RT_API int rt_group_update_camera_matrices(rt_group* g, const float inverse_projection[16],
                                           const float inverse_view[16]);
RT_API int rt_group_update_ray_directions(rt_group* g, const rt_ray* rays, uint32_t count);
RT_API int rt_group_update_spheres(rt_group* g, const rt_scene_sphere* spheres, uint32_t count);
RT_API int rt_group_update_triangles(rt_group* g, const rt_scene_triangle* triangles, uint32_t count);
RT_API int rt_group_update_object_info(rt_group* g, const rt_object_info* objects, uint32_t count);
RT_API int rt_group_update_sub_object_info(rt_group* g, const rt_sub_object_info* sub_objects, uint32_t count);
RT_API int rt_group_update_materials(rt_group* g, const rt_scene_material* materials, uint32_t count);
RT_API int rt_group_upload_textures(rt_group* g, const uint8_t* rgba8, uint32_t width, uint32_t height,
                                    uint32_t layers);
RT_API int rt_group_upload_env_map(rt_group* g, const uint8_t* rgba8, uint32_t width, uint32_t height);
/* Counted rays summed over the devices (rt_ray_count). Synchronous. */
RT_API int rt_group_ray_count(rt_group* g, uint64_t* out);
RT_API int rt_group_reset_ray_count(rt_group* g);

/* Gather payloads. */
#define RT_GATHER_IMAGE 0         /* the packed RGBA8 output, 4 B/px: the frame the reference displays */
#define RT_GATHER_ACCUMULATION 1  /* the RGBA32F accumulation, 16 B/px (+ the output rebuilt from it) */
/* Assembles the frame on device `root`: every device packs its tiles
 * (rt_pack_owned_output / rt_pack_owned_accumulation) on its stream, one grouped
 * ncclSend / ncclRecv moves every block (the root's own too) into the root's
 * receive buffer over xGMI, and the root unpacks them all in one launch
 * (rt_unpack_*_ranks; the accumulation payload re-packs the RGBA8 output with the
 * last frame's divisor k*c, compute_shader.wgsl:166). Everything is stream-ordered
 * after the frames submitted so far: the call returns without waiting for the
 * device. Afterwards the root's output (and, for RT_GATHER_ACCUMULATION, its
 * accumulation) equals a one-GPU render's; the other devices keep accumulating
 * their own tiles. */
RT_API int rt_gather_frame(rt_group* g, uint32_t root, uint32_t payload);
/* rt_read_output / rt_read_accumulation of device `root`'s context. Synchronous. */
RT_API int rt_group_read_output(rt_group* g, uint32_t root, uint32_t* rgba8_out);
RT_API int rt_group_read_accumulation(rt_group* g, uint32_t root, float* rgba_f32_out);

/* ---- scene build and edit: src/triangle_object.rs -----
 *
 * Host-side restatement of SceneObject (STL file -> placed triangles -> 7-triangle
 * sub-objects) in f32 with glam's operation order, plus the device-side
 * rebuild that Renderer::update_scene (src/renderer.rs:153-199) runs after an
 * edit. Vertices are 9 floats per triangle (a, b, c), in triangle order.
 * Calls without a context report errors through rt_last_error(NULL). */

/* The edit state of one object (SceneObject::rotation / scale /
 * transformation, src/triangle_object.rs:39-52): rotation in degrees about
 * x, y, z (applied as Rz * Ry * Rx, :253-269). 32 bytes. */
typedef struct rt_object_transform {
    float rotation[3];
    float scale;
    float transformation[3];
    uint32_t _padding;
} rt_object_transform;

/* stl_io::read_stl (src/triangle_object.rs:69): binary or ASCII STL bytes.
 * rt_stl_triangle_count gives the facet count; rt_stl_read writes 9 floats per
 * facet (normals are ignored, as in the reference). */
RT_API int rt_stl_triangle_count(const uint8_t* data, size_t size, uint32_t* count);
RT_API int rt_stl_read(const uint8_t* data, size_t size, float* vertices, uint32_t capacity);

/* SceneObject::new (src/triangle_object.rs:55-127): rotate, normalise to unit
 * diagonal, scale, drop onto the y = 0 surface, translate to `coordinates`.
 * Outputs: the normalised points the edit path starts from (9 floats per
 * triangle), the triangles (SceneTriangle::new), the ObjectInfo (bounds,
 * material; sub-object fields 0) and the initial edit state (scale 1,
 * rotation 0, transformation = coordinates + surface drop). */
RT_API int rt_scene_object_new(const float* stl_vertices, uint32_t triangle_count, float scale,
                               const float coordinates[3], const float rotation[3], uint32_t material_index,
                               float* normalized_points, rt_scene_triangle* triangles, rt_object_info* info,
                               rt_object_transform* state);

/* SceneObject::create_sub_objects (:160-197): chunks of 7 triangles with their
 * AABBs; `sub_objects` has room for ceil(triangle_count / 7). Sets the
 * object's first_sub_object_index / sub_object_count. */
RT_API int rt_scene_object_create_sub_objects(const rt_scene_triangle* triangles, uint32_t triangle_count,
                                              uint32_t first_sub_object_index, uint32_t first_triangle_index,
                                              rt_object_info* info, rt_sub_object_info* sub_objects);

/* SceneObject::update_triangles + update_sub_objects (:129-150, :199-220) on
 * the host: triangles and bounds from the normalised points and `state`.
 * `sub_objects` holds info->sub_object_count records (bounds rewritten). */
RT_API int rt_scene_object_update(const float* normalized_points, uint32_t triangle_count,
                                  const rt_object_transform* state, rt_object_info* info,
                                  rt_scene_triangle* triangles, rt_sub_object_info* sub_objects);

/* Device-side edit path. rt_set_object_models uploads every object's normalised
 * points (9 floats per triangle, in the triangle buffer's order; the objects
 * and sub-objects last set on the context say which triangles belong to which
 * object). rt_update_objects then runs update_triangles + update_sub_objects
 * for objects [0, count) on the device -- triangles, sub-object bounds,
 * object bounds -- and refits the triangle accelerator there, stream-ordered
 * before the next frame: no host round trip. Asynchronous. */
RT_API int rt_set_object_models(rt_ctx* ctx, const float* normalized_points, uint32_t triangle_count);
RT_API int rt_update_objects(rt_ctx* ctx, const rt_object_transform* transforms, uint32_t count);

/* Readback of the scene geometry the kernel sees (after host or device
 * updates). Triangles come back as full 112-byte records. Synchronous. */
RT_API int rt_read_triangles(rt_ctx* ctx, rt_scene_triangle* out, uint32_t count);
RT_API int rt_read_object_info(rt_ctx* ctx, rt_object_info* out, uint32_t count);
RT_API int rt_read_sub_object_info(rt_ctx* ctx, rt_sub_object_info* out, uint32_t count);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RT_ABI_H */
