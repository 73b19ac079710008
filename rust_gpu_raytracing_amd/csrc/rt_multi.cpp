// rt_multi.cpp — one process driving several GPUs through the C ABI
// (rt_create_multi / rt_gather_frame, include/rt_abi.h; SURVEY.md §5 "one process
// with 8 devices (ncclCommInitAll)", §8b threading row, §8e).
//
// The reference renders on one adapter from its event-loop thread
// (src/main.rs:240-496, src/renderer.rs:201-252). A group is N ordinary contexts
// -- rank r on devices[r], world N, the 8x8-tile round-robin split -- each owned
// by its own host thread, so one caller's rt_group_compute_frame enqueues the
// launches of all N GPUs concurrently (a launch costs host microseconds; eight of
// them in a row would rival an 8-way share's frame time). Rendering needs no
// communication. rt_gather_frame assembles the frame on the root with one grouped
// RCCL send/recv per rank, stream-ordered on the contexts' own streams between
// the pack and unpack kernels: no host synchronisation.
//
// RCCL is opened with dlopen on the first rt_create_multi, so single-GPU users of
// the library need neither RCCL nor its initialisation.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "rt_abi.h"

void rt_set_global_error(const std::string& msg);  // rt_abi.cpp: rt_last_error(NULL)

namespace {

// The RCCL entry points the group uses, resolved from librccl at run time.
struct Rccl {
    bool loaded = false;
    std::string error;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*get_version)(int*) = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // an RCCL already in the process (e.g. torch's) is reused by its soname
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!h) {
            r.error = std::string("cannot load librccl: ") + dlerror();
            return;
        }
        auto sym = [&](const char* n) { return dlsym(h, n); };
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(sym("ncclCommInitAll"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
        r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        r.get_version = reinterpret_cast<decltype(r.get_version)>(sym("ncclGetVersion"));
        if (!r.comm_init_all || !r.comm_destroy || !r.group_start || !r.group_end || !r.send || !r.recv ||
            !r.error_string) {
            r.error = "librccl lacks a required symbol (ncclCommInitAll/GroupStart/GroupEnd/Send/Recv)";
            return;
        }
        r.loaded = true;
    });
    return r;
}

// One device's host thread: runs the tasks posted to it, in order, on its own
// context (a context is not thread-safe; only its worker touches it while the
// group is in use).
struct Worker {
    std::thread thread;
    std::mutex m;
    std::condition_variable cv_task, cv_done;
    std::deque<std::function<int(Worker&)>> tasks;
    uint64_t posted = 0, finished = 0;
    bool stop = false;
    int first_error = RT_OK;  // the first failure of an asynchronous task, reported by the next sync call
    std::string error;
    int device = 0;
    uint32_t rank = 0;
    rt_ctx* ctx = nullptr;
    // gather buffers on this device
    void* send_buf = nullptr;
    size_t send_cap = 0;
    void* recv_buf = nullptr;  // root only: world x stride blocks
    size_t recv_cap = 0;
    // copy transport (RT_GROUP_COPY_TRANSPORT): this rank's block copied to the root on its own
    // stream (ev_sent), the root's unpack done (ev_unpacked, root only), both on this device
    hipEvent_t ev_sent = nullptr, ev_unpacked = nullptr;
    bool unpacked_recorded = false;

    void run() {
        (void)hipSetDevice(device);
        for (;;) {
            std::function<int(Worker&)> fn;
            {
                std::unique_lock<std::mutex> lk(m);
                cv_task.wait(lk, [&] { return stop || !tasks.empty(); });
                if (tasks.empty()) return;  // stop with nothing left to run
                fn = std::move(tasks.front());
                tasks.pop_front();
            }
            const int rc = fn(*this);
            std::lock_guard<std::mutex> lk(m);
            if (rc != RT_OK && first_error == RT_OK) {
                first_error = rc;
                error = "rank " + std::to_string(rank) + ": " + (ctx ? rt_last_error(ctx) : rt_last_error(nullptr));
            }
            ++finished;
            cv_done.notify_all();
        }
    }
    uint64_t post(std::function<int(Worker&)> fn) {
        std::lock_guard<std::mutex> lk(m);
        tasks.push_back(std::move(fn));
        cv_task.notify_one();
        return ++posted;
    }
    // Waits for task `ticket`; returns (and clears) the first recorded failure.
    int wait(uint64_t ticket, std::string* msg) {
        std::unique_lock<std::mutex> lk(m);
        cv_done.wait(lk, [&] { return finished >= ticket; });
        const int rc = first_error;
        if (rc != RT_OK && msg && msg->empty()) *msg = error;
        first_error = RT_OK;
        error.clear();
        return rc;
    }
};

}  // namespace

struct rt_group {
    std::vector<Worker*> workers;
    std::vector<ncclComm_t> comms;  // empty with the copy transport
    bool copy_transport = false;
    rt_params params{};  // what the contexts were last given (the gather's divisor needs compute_per_frame)
    std::string err;
};

namespace {

int group_fail(rt_group* g, int code, const std::string& msg) {
    if (g) g->err = msg; else rt_set_global_error(msg);
    return code;
}

// Runs fn(worker) on every device's thread and waits for all of them; returns
// the first failure (including failures of earlier asynchronous tasks).
int run_all(rt_group* g, const std::function<int(Worker&)>& fn) {
    g->err.clear();
    std::vector<uint64_t> t(g->workers.size());
    for (size_t i = 0; i < g->workers.size(); i++) t[i] = g->workers[i]->post(fn);
    int rc = RT_OK;
    std::string msg;
    for (size_t i = 0; i < g->workers.size(); i++) {
        const int r = g->workers[i]->wait(t[i], &msg);
        if (rc == RT_OK) rc = r;
    }
    if (rc != RT_OK) g->err = msg;
    return rc;
}

int ensure_device_buffer(Worker& w, void** buf, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *buf) return RT_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    if (hipMalloc(buf, bytes) != hipSuccess) return RT_E_NOMEM;
    *cap = bytes;
    (void)w;
    return RT_OK;
}

void destroy_group(rt_group* g) {
    if (!g) return;
    for (Worker* w : g->workers) {
        if (w->thread.joinable()) {
            w->post([](Worker& wk) {
                if (wk.ctx) (void)rt_synchronize(wk.ctx);
                if (wk.send_buf) (void)hipFree(wk.send_buf);
                if (wk.recv_buf) (void)hipFree(wk.recv_buf);
                wk.send_buf = wk.recv_buf = nullptr;
                if (wk.ev_sent) (void)hipEventDestroy(wk.ev_sent);
                if (wk.ev_unpacked) (void)hipEventDestroy(wk.ev_unpacked);
                wk.ev_sent = wk.ev_unpacked = nullptr;
                rt_destroy(wk.ctx);
                wk.ctx = nullptr;
                return RT_OK;
            });
            {
                std::lock_guard<std::mutex> lk(w->m);
                w->stop = true;
                w->cv_task.notify_one();
            }
            w->thread.join();
        }
    }
    if (!g->comms.empty() && rccl().loaded)
        for (ncclComm_t c : g->comms)
            if (c) (void)rccl().comm_destroy(c);
    for (Worker* w : g->workers) delete w;
    delete g;
}

}  // namespace

extern "C" {

int rt_create_multi(const rt_create_info* info, const int32_t* devices, uint32_t n_devices, rt_group** out) {
    return rt_create_multi_ex(info, devices, n_devices, 0u, out);
}

int rt_create_multi_ex(const rt_create_info* info, const int32_t* devices, uint32_t n_devices, uint32_t flags,
                       rt_group** out) {
    rt_set_global_error("");
    if ((flags & ~RT_GROUP_COPY_TRANSPORT) != 0u)
        return group_fail(nullptr, RT_E_INVALID, "rt_create_multi_ex: unknown flags");
    const bool copy = (flags & RT_GROUP_COPY_TRANSPORT) != 0u;
    if (!info || !devices || !out) return group_fail(nullptr, RT_E_INVALID, "rt_create_multi: NULL argument");
    *out = nullptr;
    if (n_devices == 0) return group_fail(nullptr, RT_E_INVALID, "rt_create_multi: n_devices must be >= 1");
    if (info->world_size > 1 || info->rank != 0)
        return group_fail(nullptr, RT_E_INVALID,
                          "rt_create_multi: info must describe the whole frame (rank 0, world_size 0 or 1); "
                          "the group assigns rank r to devices[r]");
    for (uint32_t i = 0; i < n_devices && !copy; i++)
        for (uint32_t j = 0; j < i; j++)
            if (devices[i] == devices[j])
                return group_fail(nullptr, RT_E_INVALID,
                                  "rt_create_multi: device " + std::to_string(devices[i]) +
                                      " listed twice (RCCL runs one rank per device)");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0)
        return group_fail(nullptr, RT_E_NODEVICE, "no HIP device available");
    for (uint32_t i = 0; i < n_devices; i++)
        if (devices[i] < 0 || devices[i] >= n_dev)
            return group_fail(nullptr, RT_E_NODEVICE, "rt_create_multi: device ordinal out of range");
    if (!copy && !rccl().loaded) return group_fail(nullptr, RT_E_NODEVICE, "rt_create_multi: " + rccl().error);

    rt_group* g = new (std::nothrow) rt_group();
    if (!g) return group_fail(nullptr, RT_E_NOMEM, "out of host memory");
    g->params = info->params;
    g->copy_transport = copy;
    for (uint32_t r = 0; r < n_devices; r++) {
        Worker* w = new (std::nothrow) Worker();
        if (!w) {
            destroy_group(g);
            return group_fail(nullptr, RT_E_NOMEM, "out of host memory");
        }
        w->device = devices[r];
        w->rank = r;
        g->workers.push_back(w);
        w->thread = std::thread([w] { w->run(); });
    }
    // every context is created on its own thread, in parallel (uploads of the
    // scene, camera rays and later textures run concurrently on the N devices)
    const rt_create_info base = *info;
    int rc = run_all(g, [base, n_devices](Worker& w) {
        rt_create_info ci = base;
        ci.device = w.device;
        ci.rank = w.rank;
        ci.world_size = n_devices;
        return rt_create(&ci, &w.ctx);
    });
    if (rc != RT_OK) {
        const std::string msg = g->err;
        destroy_group(g);
        return group_fail(nullptr, rc, "rt_create_multi: " + msg);
    }
    if (copy) {  // no communicators: the gather copies blocks device to device
        *out = g;
        return RT_OK;
    }
    // one communicator per device, in this process
    Rccl& R = rccl();
    g->comms.assign(n_devices, nullptr);
    std::vector<int> devlist(devices, devices + n_devices);
    const ncclResult_t nr = R.comm_init_all(g->comms.data(), (int)n_devices, devlist.data());
    if (nr != ncclSuccess) {
        const std::string msg = R.error_string(nr);
        g->comms.assign(n_devices, nullptr);
        destroy_group(g);
        return group_fail(nullptr, RT_E_HIP, std::string("ncclCommInitAll: ") + msg);
    }
    *out = g;
    return RT_OK;
}

void rt_destroy_multi(rt_group* g) { destroy_group(g); }

const char* rt_group_last_error(const rt_group* g) { return g ? g->err.c_str() : rt_last_error(nullptr); }

uint32_t rt_group_size(const rt_group* g) { return g ? (uint32_t)g->workers.size() : 0u; }

rt_ctx* rt_group_context(rt_group* g, uint32_t rank) {
    if (!g || rank >= g->workers.size()) return nullptr;
    return g->workers[rank]->ctx;
}

int rt_group_compute_frame(rt_group* g, uint32_t bounces) {
    if (!g) return RT_E_INVALID;
    g->err.clear();
    // asynchronous: each device's thread queues (or launches) its share; a failure
    // is reported by the next synchronous group call
    for (Worker* w : g->workers) w->post([bounces](Worker& wk) { return rt_compute_frame(wk.ctx, bounces); });
    return RT_OK;
}

int rt_group_synchronize(rt_group* g) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [](Worker& w) { return rt_synchronize(w.ctx); });
}

int rt_group_flush(rt_group* g) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [](Worker& w) { return rt_flush(w.ctx); });
}

int rt_group_set_frame_batch(rt_group* g, uint32_t max_frames) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [max_frames](Worker& w) { return rt_set_frame_batch(w.ctx, max_frames); });
}

int rt_group_update_params(rt_group* g, const rt_params* params) {
    if (!g || !params) return g ? group_fail(g, RT_E_INVALID, "params is NULL") : RT_E_INVALID;
    const rt_params p = *params;
    const int rc = run_all(g, [p](Worker& w) { return rt_update_params(w.ctx, &p); });
    if (rc == RT_OK) g->params = p;
    return rc;
}

int rt_group_reset_accumulation(rt_group* g, const rt_params* params) {
    if (!g || !params) return g ? group_fail(g, RT_E_INVALID, "params is NULL") : RT_E_INVALID;
    const rt_params p = *params;
    const int rc = run_all(g, [p](Worker& w) { return rt_reset_accumulation(w.ctx, &p); });
    if (rc == RT_OK) g->params = p;
    return rc;
}

int rt_group_update_camera(rt_group* g, const rt_ray_camera* camera) {
    if (!g || !camera) return g ? group_fail(g, RT_E_INVALID, "camera is NULL") : RT_E_INVALID;
    const rt_ray_camera c = *camera;
    return run_all(g, [c](Worker& w) { return rt_update_camera(w.ctx, &c); });
}

int rt_group_update_camera_matrices(rt_group* g, const float inverse_projection[16], const float inverse_view[16]) {
    if (!g || !inverse_projection || !inverse_view)
        return g ? group_fail(g, RT_E_INVALID, "matrix is NULL") : RT_E_INVALID;
    return run_all(g, [=](Worker& w) { return rt_update_camera_matrices(w.ctx, inverse_projection, inverse_view); });
}

// Host arrays are read by every device's thread; the call returns once all of
// them have copied the data (rt_update_* copy before returning), so the caller
// keeps ownership exactly as with one context.
#define RT_GROUP_UPDATE(NAME, TYPE)                                                     \
    int rt_group_##NAME(rt_group* g, const TYPE* data, uint32_t count) {               \
        if (!g) return RT_E_INVALID;                                                    \
        return run_all(g, [=](Worker& w) { return rt_##NAME(w.ctx, data, count); }); \
    }
RT_GROUP_UPDATE(update_ray_directions, rt_ray)
RT_GROUP_UPDATE(update_spheres, rt_scene_sphere)
RT_GROUP_UPDATE(update_triangles, rt_scene_triangle)
RT_GROUP_UPDATE(update_object_info, rt_object_info)
RT_GROUP_UPDATE(update_sub_object_info, rt_sub_object_info)
RT_GROUP_UPDATE(update_materials, rt_scene_material)
#undef RT_GROUP_UPDATE

int rt_group_upload_textures(rt_group* g, const uint8_t* rgba8, uint32_t width, uint32_t height, uint32_t layers) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [=](Worker& w) { return rt_upload_textures(w.ctx, rgba8, width, height, layers); });
}

int rt_group_upload_env_map(rt_group* g, const uint8_t* rgba8, uint32_t width, uint32_t height) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [=](Worker& w) { return rt_upload_env_map(w.ctx, rgba8, width, height); });
}

int rt_group_ray_count(rt_group* g, uint64_t* out) {
    if (!g || !out) return g ? group_fail(g, RT_E_INVALID, "out is NULL") : RT_E_INVALID;
    std::vector<uint64_t> n(g->workers.size(), 0);
    const int rc = run_all(g, [&n](Worker& w) { return rt_ray_count(w.ctx, &n[w.rank]); });
    uint64_t s = 0;
    for (uint64_t v : n) s += v;
    *out = s;
    return rc;
}

int rt_group_reset_ray_count(rt_group* g) {
    if (!g) return RT_E_INVALID;
    return run_all(g, [](Worker& w) { return rt_reset_ray_count(w.ctx); });
}

int rt_gather_frame(rt_group* g, uint32_t root, uint32_t payload) {
    if (!g) return RT_E_INVALID;
    g->err.clear();
    const uint32_t n = (uint32_t)g->workers.size();
    if (root >= n) return group_fail(g, RT_E_INVALID, "rt_gather_frame: root out of range");
    if (payload != RT_GATHER_IMAGE && payload != RT_GATHER_ACCUMULATION)
        return group_fail(g, RT_E_INVALID, "rt_gather_frame: payload must be RT_GATHER_IMAGE or RT_GATHER_ACCUMULATION");
    if (payload == RT_GATHER_ACCUMULATION && g->params.accumulate != 1)
        return group_fail(g, RT_E_INVALID,
                          "rt_gather_frame: a non-accumulating render never writes its accumulation "
                          "(compute_shader.wgsl:171-178); gather the image");
    const size_t px_bytes = payload == RT_GATHER_IMAGE ? 4 : 16;
    // every block padded to rank 0's (the largest) pixel count
    uint64_t stride_px = 0;
    if (rt_owned_pixel_count(g->workers[0]->ctx, 0, n, &stride_px) != RT_OK)
        return group_fail(g, RT_E_INVALID, "rt_gather_frame: bad context");
    const size_t block = (size_t)stride_px * px_bytes;
    Worker* rw = g->workers[root];
    const bool copy = g->copy_transport;
    // 0. buffers (the root's receive slots must exist before another rank copies into them)
    int rc = run_all(g, [&](Worker& w) {
        int r = ensure_device_buffer(w, &w.send_buf, &w.send_cap, block);
        if (r == RT_OK && w.rank == root) r = ensure_device_buffer(w, &w.recv_buf, &w.recv_cap, block * n);
        if (r == RT_OK && copy) {
            if (!w.ev_sent && hipEventCreateWithFlags(&w.ev_sent, hipEventDisableTiming) != hipSuccess) r = RT_E_HIP;
            if (!w.ev_unpacked && hipEventCreateWithFlags(&w.ev_unpacked, hipEventDisableTiming) != hipSuccess)
                r = RT_E_HIP;
        }
        return r;
    });
    if (rc != RT_OK) return rc;
    // 1. on every device: queued frames launched, its tiles packed on its stream (copy
    // transport: then copied into slot r of the root's receive buffer on the same stream,
    // once the root has unpacked the previous gather out of it)
    std::vector<hipStream_t> streams(n, nullptr);
    uint8_t* const recv = static_cast<uint8_t*>(rw->recv_buf);
    const int root_dev = rw->device;
    hipEvent_t const prev_unpacked = rw->unpacked_recorded ? rw->ev_unpacked : nullptr;
    rc = run_all(g, [&](Worker& w) {
        int r = payload == RT_GATHER_IMAGE ? rt_pack_owned_output(w.ctx, w.send_buf)
                                           : rt_pack_owned_accumulation(w.ctx, w.send_buf);
        if (r != RT_OK) return r;
        hipStream_t s = static_cast<hipStream_t>(rt_stream(w.ctx));
        streams[w.rank] = s;
        if (!s) return RT_E_HIP;
        if (copy) {
            if (prev_unpacked && hipStreamWaitEvent(s, prev_unpacked, 0) != hipSuccess) return RT_E_HIP;
            if (hipMemcpyPeerAsync(recv + (size_t)w.rank * block, root_dev, w.send_buf, w.device, block, s) !=
                    hipSuccess ||
                hipEventRecord(w.ev_sent, s) != hipSuccess)
                return RT_E_HIP;
        }
        return RT_OK;
    });
    if (rc != RT_OK) return rc;
    if (copy) {
        // 3. the root waits for every copy, unpacks every block, and marks its receive
        // buffer free for the next gather's copies
        uint32_t k = 1;
        (void)rt_accumulation_index(rw->ctx, &k);
        const uint32_t divisor = std::max<uint32_t>(k - 1, 1) * std::max<uint32_t>(g->params.compute_per_frame, 1);
        std::vector<hipEvent_t> sent(n);
        for (uint32_t r = 0; r < n; r++) sent[r] = g->workers[r]->ev_sent;
        const uint64_t t = rw->post([=](Worker& w) {
            hipStream_t s = static_cast<hipStream_t>(rt_stream(w.ctx));
            for (hipEvent_t ev : sent)
                if (hipStreamWaitEvent(s, ev, 0) != hipSuccess) return (int)RT_E_HIP;
            const int r = payload == RT_GATHER_IMAGE ? rt_unpack_output_ranks(w.ctx, w.recv_buf, stride_px, n, n)
                                                     : rt_unpack_accumulation_ranks(w.ctx, w.recv_buf, stride_px, n,
                                                                                    n, divisor);
            if (r != RT_OK) return r;
            if (hipEventRecord(w.ev_unpacked, s) != hipSuccess) return (int)RT_E_HIP;
            w.unpacked_recorded = true;
            return (int)RT_OK;
        });
        std::string msg;
        rc = rw->wait(t, &msg);
        if (rc != RT_OK) g->err = msg.empty() ? "rt_gather_frame: copy transport failed" : msg;
        return rc;
    }
    Rccl& R = rccl();
    // 2. one grouped send/recv: rank r's block to slot r of the root's buffer
    // (the root's own block too, a local copy: one unpack launch then covers every
    // block, and a one-GPU group moves its data through RCCL like any other)
    if (R.group_start() != ncclSuccess) return group_fail(g, RT_E_HIP, "ncclGroupStart failed");
    ncclResult_t nr = ncclSuccess;
    for (uint32_t r = 0; r < n && nr == ncclSuccess; r++) {
        Worker* w = g->workers[r];
        nr = R.send(w->send_buf, block, ncclUint8, (int)root, g->comms[r], streams[r]);
        if (nr == ncclSuccess)
            nr = R.recv(static_cast<uint8_t*>(rw->recv_buf) + (size_t)r * block, block, ncclUint8, (int)r,
                        g->comms[root], streams[root]);
    }
    const ncclResult_t ne = R.group_end();
    if (nr == ncclSuccess) nr = ne;
    if (nr != ncclSuccess) return group_fail(g, RT_E_HIP, std::string("RCCL gather: ") + R.error_string(nr));
    // 3. the root unpacks every block, stream-ordered after its receives
    uint32_t k = 1;
    (void)rt_accumulation_index(rw->ctx, &k);
    const uint32_t divisor = std::max<uint32_t>(k - 1, 1) * std::max<uint32_t>(g->params.compute_per_frame, 1);
    const uint64_t t = rw->post([=](Worker& w) {
        return payload == RT_GATHER_IMAGE ? rt_unpack_output_ranks(w.ctx, w.recv_buf, stride_px, n, n)
                                          : rt_unpack_accumulation_ranks(w.ctx, w.recv_buf, stride_px, n, n, divisor);
    });
    std::string msg;
    rc = rw->wait(t, &msg);
    if (rc != RT_OK) g->err = msg;
    return rc;
}

int rt_group_read_output(rt_group* g, uint32_t root, uint32_t* rgba8_out) {
    if (!g || !rgba8_out || root >= g->workers.size())
        return g ? group_fail(g, RT_E_INVALID, "rt_group_read_output: bad argument") : RT_E_INVALID;
    Worker* w = g->workers[root];
    std::string msg;
    const int rc = w->wait(w->post([rgba8_out](Worker& wk) { return rt_read_output(wk.ctx, rgba8_out); }), &msg);
    if (rc != RT_OK) g->err = msg;
    return rc;
}

int rt_group_read_accumulation(rt_group* g, uint32_t root, float* rgba_f32_out) {
    if (!g || !rgba_f32_out || root >= g->workers.size())
        return g ? group_fail(g, RT_E_INVALID, "rt_group_read_accumulation: bad argument") : RT_E_INVALID;
    Worker* w = g->workers[root];
    std::string msg;
    const int rc =
        w->wait(w->post([rgba_f32_out](Worker& wk) { return rt_read_accumulation(wk.ctx, rgba_f32_out); }), &msg);
    if (rc != RT_OK) g->err = msg;
    return rc;
}

}  // extern "C"
