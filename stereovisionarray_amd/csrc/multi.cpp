// multi.cpp -- multi-pair / multi-GPU host layer of libsva.so (include/sva.h,
// "multi-pair batch" and "multi-GPU engine").
//
// Host C++ only.  Pairs are the shard unit: pair j -> device j mod N and
// round-robin over that device's contexts (one HIP stream each), so each
// device keeps its own cost / path volumes and nothing crosses devices until
// the finished u16 disparity maps (and optional f32 sub-pixel maps) are
// gathered to devices[0] -- an RCCL grouped send/recv on a single-process
// communicator (ncclCommInitAll over the engine's devices; librccl is opened
// at sva_multi_create, so libsva.so itself has no RCCL link dependency), or
// peer copies over xGMI (SVA_MULTI_GATHER_PEER).  Every compute step goes
// through the public per-context entry points (sva_disparity_sgm_d,
// sva_fuse_depth_d); there is no CPU path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "sva_internal.h"

using namespace sva;

namespace {

// ------------------------------------------------------------ pinned host --
struct PinnedBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes && ptr) return hipSuccess;
        release();
        hipError_t e = hipHostMalloc(&ptr, std::max<size_t>(n, 256), hipHostMallocDefault);
        if (e != hipSuccess) { ptr = nullptr; return e; }
        bytes = std::max<size_t>(n, 256);
        return hipSuccess;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

void copy_plane(uint8_t* dst, const uint8_t* src, int W, int H, size_t pitch) {
    if (pitch == (size_t)W) {
        std::memcpy(dst, src, (size_t)W * H);
        return;
    }
    for (int y = 0; y < H; y++) std::memcpy(dst + (size_t)y * W, src + (size_t)y * pitch, W);
}

// ------------------------------------------------------------------ RCCL --
// The few RCCL entry points the gather uses, resolved from librccl.so.1.
struct Rccl {
    void* lib = nullptr;
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;

    bool open(std::string& err) {
        const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        for (const char* n : names)
            if ((lib = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!lib) {
            err = "cannot load librccl.so.1 (RCCL gather); use SVA_MULTI_GATHER_PEER";
            return false;
        }
#define SVA_SYM(field, name)                                                   \
    field = reinterpret_cast<decltype(field)>(dlsym(lib, name));               \
    if (!field) { err = std::string("librccl lacks ") + name; return false; }
        SVA_SYM(commInitAll, "ncclCommInitAll");
        SVA_SYM(commDestroy, "ncclCommDestroy");
        SVA_SYM(groupStart, "ncclGroupStart");
        SVA_SYM(groupEnd, "ncclGroupEnd");
        SVA_SYM(send, "ncclSend");
        SVA_SYM(recv, "ncclRecv");
        SVA_SYM(errorString, "ncclGetErrorString");
#undef SVA_SYM
        return true;
    }
};

// ---------------------------------------------------------------- engine --
struct Multi {
    std::vector<int> devices;
    int spd = 1;                       // streams (contexts) per device
    int mode = SVA_MULTI_GATHER_RCCL;
    bool gather_all = false;
    std::vector<void*> ctx;            // [d * spd + s]
    std::vector<hipStream_t> copy;     // per device: uploads
    std::vector<hipStream_t> down;     // per device: downloads (device 0 used)
    std::vector<hipEvent_t> gathered;  // per device: last gather done (slot reuse), re-recorded
    bool gathered_valid = false;
    std::vector<std::vector<hipEvent_t>> ev_all;   // per device: per-call events, recycled
    std::vector<size_t> ev_used;
    std::vector<DevBuf> slots;         // per context: local maps of gathered jobs
    std::vector<DevBuf> images;        // per device: uploaded views (sva_array_depth)
    DevBuf maps0, depth0, nvalid0;     // device 0 (sva_array_depth)
    PinnedBuf stage_in, stage_out;
    Rccl rccl;
    std::vector<ncclComm_t> comms;
    std::string last_error;

    int nd() const { return (int)devices.size(); }
    Ctx* c(int d, int s) const { return static_cast<Ctx*>(ctx[(size_t)d * spd + s]); }
    hipStream_t st(int d, int s) const { return c(d, s)->stream; }

    int fail(int code, const std::string& m) {
        last_error = m;
        return code;
    }
    int hip_fail(hipError_t e, const char* what) {
        last_error = std::string(what) + ": " + hipGetErrorString(e);
        return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? SVA_ERR_OUT_OF_MEMORY
                                                                          : SVA_ERR_DEVICE;
    }
    int ctx_fail(int code, void* cx, const char* what) {
        last_error = std::string(what) + ": " + sva_last_error(cx);
        return code;
    }
};

#define MHIP(m, expr, what)                                  \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return (m)->hip_fail(_e, what); \
    } while (0)

Multi* as_multi(void* p) { return static_cast<Multi*>(p); }

// A per-call event recorded on device d (recorded events must belong to the
// recording stream's device; any device's stream may wait on them).  Pools are
// reset at the start of each call: a stream wait already enqueued keeps the
// record it captured, so re-recording an event later is safe.
hipError_t ev_on(Multi* m, int d, hipEvent_t* out) {
    hipError_t e = hipSetDevice(m->devices[d]);
    if (e != hipSuccess) return e;
    if (m->ev_used[d] < m->ev_all[d].size()) {
        *out = m->ev_all[d][m->ev_used[d]++];
        return hipSuccess;
    }
    hipEvent_t ev;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    m->ev_all[d].push_back(ev);
    m->ev_used[d]++;
    *out = ev;
    return hipSuccess;
}
void ev_reset(Multi* m) { std::fill(m->ev_used.begin(), m->ev_used.end(), 0); }

// `waiter` (on device dw) waits for everything queued so far on `src` (device ds).
int stream_after(Multi* m, int ds, hipStream_t src, hipStream_t waiter) {
    hipEvent_t e;
    MHIP(m, ev_on(m, ds, &e), "event");
    MHIP(m, hipEventRecord(e, src), "event record");
    MHIP(m, hipStreamWaitEvent(waiter, e, 0), "stream wait");
    return SVA_OK;
}

struct Plan {
    std::vector<int32_t> dev, cx, slot;
    std::vector<int> per_ctx;   // jobs per context
};

void make_plan(int nd, int spd, int n, Plan& p) {
    p.dev.resize(n);
    p.cx.resize(n);
    p.slot.resize(n);
    p.per_ctx.assign((size_t)nd * spd, 0);
    for (int j = 0; j < n; j++) {
        p.dev[j] = j % nd;
        p.cx[j] = (j / nd) % spd;
        p.slot[j] = p.per_ctx[(size_t)p.dev[j] * spd + p.cx[j]]++;
    }
}

// Gather job maps living in per-context slots to `dst` on devices[0]:
// dst + j*bytes  <-  slot(j).  `remote[j]` says whether job j needs it.
// All contexts' streams of each device have been joined into st(d, 0).
int gather(Multi* m, const Plan& P, const std::vector<char>& remote,
           const std::vector<const uint8_t*>& src, uint8_t* dst, size_t bytes) {
    const int n = (int)P.dev.size();
    if (m->mode == SVA_MULTI_GATHER_RCCL) {
        ncclResult_t r = m->rccl.groupStart();
        if (r != ncclSuccess) return m->fail(SVA_ERR_DEVICE, m->rccl.errorString(r));
        for (int j = 0; j < n; j++) {
            if (!remote[j]) continue;
            const int d = P.dev[j];
            r = m->rccl.send(src[j], bytes, ncclUint8, 0, m->comms[d], m->st(d, 0));
            if (r == ncclSuccess)
                r = m->rccl.recv(dst + (size_t)j * bytes, bytes, ncclUint8, d, m->comms[0],
                                 m->st(0, 0));
            if (r != ncclSuccess) {
                (void)m->rccl.groupEnd();
                return m->fail(SVA_ERR_DEVICE, std::string("RCCL: ") + m->rccl.errorString(r));
            }
        }
        r = m->rccl.groupEnd();
        if (r != ncclSuccess)
            return m->fail(SVA_ERR_DEVICE, std::string("RCCL: ") + m->rccl.errorString(r));
        return SVA_OK;
    }
    // peer copies, issued on the source device's stream; device 0 joins them
    std::vector<char> used(m->nd(), 0);
    for (int j = 0; j < n; j++) {
        if (!remote[j]) continue;
        const int d = P.dev[j];
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        MHIP(m, hipMemcpyAsync(dst + (size_t)j * bytes, src[j], bytes, hipMemcpyDeviceToDevice,
                               m->st(d, 0)),
             "peer copy");
        used[d] = 1;
    }
    for (int d = 1; d < m->nd(); d++)
        if (used[d]) {
            int s = stream_after(m, d, m->st(d, 0), m->st(0, 0));
            if (s) return s;
        }
    return SVA_OK;
}

// The shared part of sva_batch_sgm_d / sva_array_depth: run every pair on its
// context, gather to devices[0].  left/right: per-job device pointers;
// maps/sub on devices[0] ([n][H][W]); sub may be null.
int run_pairs(Multi* m, const Plan& P, const std::vector<const uint8_t*>& left,
              const std::vector<const uint8_t*>& right, const std::vector<sva_sgm_params>& prm,
              const std::vector<std::vector<hipEvent_t>>& wait_for, int W, int H, size_t pitch,
              uint16_t* maps, float* sub) {
    const int n = (int)P.dev.size();
    const size_t np = (size_t)W * H;
    // 0. maps / sub are the caller's buffers on devices[0]: results of the
    // previous call are complete on st(0, 0), and the caller may still be
    // reading them there.  Every stream that writes into maps / sub -- device
    // 0's other context streams (local jobs) and, with peer copies, each source
    // device's st(d, 0) -- starts after what is queued on st(0, 0) now.  (The
    // RCCL receives run on st(0, 0) itself.)
    {
        hipEvent_t e0;
        MHIP(m, ev_on(m, 0, &e0), "event");
        MHIP(m, hipEventRecord(e0, m->st(0, 0)), "event record");
        for (int s = 1; s < m->spd; s++)
            MHIP(m, hipStreamWaitEvent(m->st(0, s), e0, 0), "stream wait");
        if (m->mode == SVA_MULTI_GATHER_PEER)
            for (int d = 1; d < m->nd(); d++) {
                MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
                MHIP(m, hipStreamWaitEvent(m->st(d, 0), e0, 0), "stream wait");
            }
    }
    // 1. slot workspace per context; a context starts after its device's last gather
    std::vector<char> remote(n, 0);
    for (int j = 0; j < n; j++) remote[j] = P.dev[j] != 0 || m->gather_all;
    const size_t per = np * 2 + (sub ? np * 4 : 0);
    for (int d = 0; d < m->nd(); d++) {
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        for (int s = 0; s < m->spd; s++) {
            const size_t ci = (size_t)d * m->spd + s;
            if (P.per_ctx[ci] == 0) continue;
            if (d != 0 || m->gather_all) MHIP(m, m->slots[ci].ensure(per * P.per_ctx[ci]), "slots");
            if (m->gathered_valid)
                MHIP(m, hipStreamWaitEvent(m->st(d, s), m->gathered[d], 0), "wait");
        }
    }
    // 2. compute
    std::vector<const uint8_t*> src_map(n, nullptr), src_sub(n, nullptr);
    for (int j = 0; j < n; j++) {
        const int d = P.dev[j], s = P.cx[j];
        const size_t ci = (size_t)d * m->spd + s;
        uint16_t* od;
        float* os = nullptr;
        if (remote[j]) {
            uint8_t* base = (uint8_t*)m->slots[ci].ptr + (size_t)P.slot[j] * per;
            od = (uint16_t*)base;
            if (sub) os = (float*)(base + np * 2);
            src_map[j] = base;
            src_sub[j] = base + np * 2;
        } else {
            od = maps + (size_t)j * np;
            if (sub) os = sub + (size_t)j * np;
        }
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        for (hipEvent_t e : wait_for[j]) MHIP(m, hipStreamWaitEvent(m->st(d, s), e, 0), "wait");
        const int st = sva_disparity_sgm_d(m->ctx[ci], left[j], right[j], W, H, pitch, &prm[j], od,
                                           os);
        if (st != SVA_OK) return m->ctx_fail(st, m->ctx[ci], "pair");
    }
    // 3. join each device's streams into its stream 0
    for (int d = 0; d < m->nd(); d++)
        for (int s = 1; s < m->spd; s++) {
            if (P.per_ctx[(size_t)d * m->spd + s] == 0) continue;
            int st = stream_after(m, d, m->st(d, s), m->st(d, 0));
            if (st) return st;
        }
    // 4. gather (maps, then sub-pixel maps)
    int st = gather(m, P, remote, src_map, (uint8_t*)maps, np * 2);
    if (st) return st;
    if (sub) {
        // only jobs that asked for a sub-pixel map have one (sva.h); the
        // others' planes of `sub` are left untouched, local or remote
        std::vector<char> remote_sub(remote);
        for (int j = 0; j < n; j++) remote_sub[j] = remote[j] && prm[j].subpixel != 0;
        if ((st = gather(m, P, remote_sub, src_sub, (uint8_t*)sub, np * 4))) return st;
    }
    for (int d = 0; d < m->nd(); d++) {
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        MHIP(m, hipEventRecord(m->gathered[d], m->st(d, 0)), "event record");
    }
    m->gathered_valid = true;
    return SVA_OK;
}

int check_params(const sva_sgm_params& p) {
    if (!padded_D(p.D) || p.dmin < 0 || (p.dir == 0 && p.dir_y == 0))
        return SVA_ERR_INVALID_ARG;
    return SVA_OK;
}

// ------------------------------------------- host batch (sva_batch_sgm) --
// One context's share of sva_batch_sgm: jobs i, i + n, ...; two pipeline
// slots so that upload(j+1) / download(j-1) overlap compute(j).  The lane
// (streams, events, pinned and device staging) lives in the context
// (Ctx::batch_lane) from its first batch to sva_destroy: hipHostMalloc /
// hipFree synchronise the device, so a lane per call cost milliseconds.
struct HostLane {
    Ctx* c = nullptr;
    hipStream_t up = nullptr, dn = nullptr;
    PinnedBuf in[2], out[2];
    DevBuf din[2], dout[2];
    hipEvent_t e_up[2] = {}, e_comp[2] = {}, e_dn[2] = {};
    int job[2] = {-1, -1};
};

int lane_init(HostLane& L) {
    if (hipSetDevice(L.c->device) != hipSuccess) return SVA_ERR_DEVICE;
    if (hipStreamCreateWithFlags(&L.up, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&L.dn, hipStreamNonBlocking) != hipSuccess)
        return SVA_ERR_DEVICE;
    for (int b = 0; b < 2; b++)
        if (hipEventCreateWithFlags(&L.e_up[b], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.e_comp[b], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.e_dn[b], hipEventDisableTiming) != hipSuccess)
            return SVA_ERR_DEVICE;
    return SVA_OK;
}

void lane_free(HostLane& L) {
    (void)hipSetDevice(L.c->device);
    if (L.up) (void)hipStreamSynchronize(L.up);
    if (L.dn) (void)hipStreamSynchronize(L.dn);
    for (int b = 0; b < 2; b++) {
        L.in[b].release();
        L.out[b].release();
        L.din[b].release();
        L.dout[b].release();
        for (hipEvent_t e : {L.e_up[b], L.e_comp[b], L.e_dn[b]})
            if (e) (void)hipEventDestroy(e);
    }
    if (L.up) (void)hipStreamDestroy(L.up);
    if (L.dn) (void)hipStreamDestroy(L.dn);
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- batch --
int sva_batch_sgm(void** ctxs, int n_ctx, const sva_pair_job* jobs, int n_jobs,
                  const sva_sgm_params* p, int* job_status) {
    if (!ctxs || n_ctx <= 0 || (n_jobs > 0 && !jobs) || n_jobs < 0 || !p)
        return SVA_ERR_INVALID_ARG;
    for (int i = 0; i < n_ctx; i++) {
        if (!ctxs[i]) return SVA_ERR_INVALID_ARG;
        for (int k = 0; k < i; k++)
            if (ctxs[k] == ctxs[i]) return SVA_ERR_INVALID_ARG;   // a context is not re-entrant
    }
    std::vector<int> status(n_jobs, SVA_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n_ctx; i++) {
        th.emplace_back([&, i]() {
            Ctx* cx = static_cast<Ctx*>(ctxs[i]);
            int s0 = SVA_OK;
            if (!cx->batch_lane) {
                HostLane* nl = new (std::nothrow) HostLane();
                if (!nl) {
                    s0 = SVA_ERR_OUT_OF_MEMORY;
                } else {
                    nl->c = cx;
                    s0 = lane_init(*nl);
                    cx->batch_lane = std::shared_ptr<void>(nl, [](void* q) {
                        HostLane* h = static_cast<HostLane*>(q);
                        lane_free(*h);
                        delete h;
                    });
                    if (s0 != SVA_OK) cx->batch_lane.reset();
                }
            }
            HostLane dummy;
            HostLane& L = cx->batch_lane ? *static_cast<HostLane*>(cx->batch_lane.get()) : dummy;
            L.job[0] = L.job[1] = -1;
            // finish job in slot b: wait for its download, copy out of pinned memory
            auto finish = [&](int b) {
                const int j = L.job[b];
                if (j < 0) return;
                L.job[b] = -1;
                if (hipEventSynchronize(L.e_dn[b]) != hipSuccess) {
                    status[j] = SVA_ERR_DEVICE;
                    return;
                }
                const sva_pair_job& J = jobs[j];
                const size_t np = (size_t)J.width * J.height;
                std::memcpy(J.disp, L.out[b].ptr, np * 2);
                if (J.subpix && p->subpixel)
                    std::memcpy(J.subpix, (uint8_t*)L.out[b].ptr + np * 2, np * 4);
            };
            int q = 0;
            for (int j = i; j < n_jobs; j += n_ctx, q++) {
                if (s0 != SVA_OK) { status[j] = s0; continue; }
                const int b = q & 1;
                finish(b);                                   // job q-2 frees slot b
                const sva_pair_job& J = jobs[j];
                if (!J.left || !J.right || !J.disp || J.width <= 0 || J.height <= 0 ||
                    J.pitch < (size_t)J.width) {
                    status[j] = SVA_ERR_INVALID_ARG;
                    continue;
                }
                const int W = J.width, H = J.height;
                const size_t np = (size_t)W * H;
                const bool want_sub = J.subpix && p->subpixel;
                const size_t out_bytes = np * 2 + (want_sub ? np * 4 : 0);
                if (L.in[b].ensure(np * 2) != hipSuccess ||
                    L.out[b].ensure(out_bytes) != hipSuccess ||
                    L.din[b].ensure(np * 2) != hipSuccess ||
                    L.dout[b].ensure(out_bytes) != hipSuccess) {
                    status[j] = SVA_ERR_OUT_OF_MEMORY;
                    continue;
                }
                uint8_t* pin = (uint8_t*)L.in[b].ptr;
                copy_plane(pin, J.left, W, H, J.pitch);
                copy_plane(pin + np, J.right, W, H, J.pitch);
                uint8_t* d_in = (uint8_t*)L.din[b].ptr;
                uint8_t* d_out = (uint8_t*)L.dout[b].ptr;
                hipError_t e = hipMemcpyAsync(d_in, pin, np * 2, hipMemcpyHostToDevice, L.up);
                if (e == hipSuccess) e = hipEventRecord(L.e_up[b], L.up);
                if (e == hipSuccess) e = hipStreamWaitEvent(L.c->stream, L.e_up[b], 0);
                if (e != hipSuccess) { status[j] = SVA_ERR_DEVICE; continue; }
                const int st = sva_disparity_sgm_d(L.c, d_in, d_in + np, W, H, W, p,
                                                   (uint16_t*)d_out,
                                                   want_sub ? (float*)(d_out + np * 2) : nullptr);
                if (st != SVA_OK) {
                    status[j] = st;
                    (void)hipStreamSynchronize(L.c->stream);
                    continue;
                }
                e = hipEventRecord(L.e_comp[b], L.c->stream);
                if (e == hipSuccess) e = hipStreamWaitEvent(L.dn, L.e_comp[b], 0);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(L.out[b].ptr, d_out, out_bytes, hipMemcpyDeviceToHost, L.dn);
                if (e == hipSuccess) e = hipEventRecord(L.e_dn[b], L.dn);
                if (e != hipSuccess) { status[j] = SVA_ERR_DEVICE; continue; }
                L.job[b] = j;
                // the upload of the next job reuses pinned slot b^1 only after
                // finish(b^1), which waits for that slot's download
            }
            finish(0);
            finish(1);
            // pinned input slots are reused only after their upload completed:
            // e_up precedes e_comp precedes e_dn, which finish() waited on
        });
    }
    for (auto& t : th) t.join();
    int first = SVA_OK;
    for (int j = 0; j < n_jobs; j++) {
        if (job_status) job_status[j] = status[j];
        if (first == SVA_OK && status[j] != SVA_OK) first = status[j];
    }
    return first;
}

// ---------------------------------------------------------------- multi --
int sva_multi_plan(int n_devices, int spd, int n_jobs, int32_t* device_index,
                   int32_t* context_index, int32_t* slot_index) {
    if (n_devices <= 0 || spd <= 0 || n_jobs < 0) return SVA_ERR_INVALID_ARG;
    Plan P;
    make_plan(n_devices, spd, n_jobs, P);
    for (int j = 0; j < n_jobs; j++) {
        if (device_index) device_index[j] = P.dev[j];
        if (context_index) context_index[j] = P.cx[j];
        if (slot_index) slot_index[j] = P.slot[j];
    }
    return SVA_OK;
}

int sva_multi_create(const int* devices, int n_devices, int spd, int flags, void** out) {
    if (!devices || n_devices <= 0 || spd <= 0 || spd > 8 || !out || (flags & ~3))
        return SVA_ERR_INVALID_ARG;
    const int mode = flags & 1;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SVA_ERR_NO_DEVICE;
    for (int i = 0; i < n_devices; i++) {
        if (devices[i] < 0 || devices[i] >= count) return SVA_ERR_INVALID_ARG;
        for (int k = 0; k < i; k++)
            if (devices[k] == devices[i]) return SVA_ERR_INVALID_ARG;   // one rank per GPU
    }
    Multi* m = new (std::nothrow) Multi();
    if (!m) return SVA_ERR_OUT_OF_MEMORY;
    m->devices.assign(devices, devices + n_devices);
    m->spd = spd;
    m->mode = mode;
    m->gather_all = (flags & SVA_MULTI_GATHER_ALL) != 0;
    m->ctx.assign((size_t)n_devices * spd, nullptr);
    m->slots.resize((size_t)n_devices * spd);
    m->images.resize(n_devices);
    m->gathered.assign(n_devices, nullptr);
    m->ev_all.resize(n_devices);
    m->ev_used.assign(n_devices, 0);
    int st = SVA_OK;
    for (int d = 0; d < n_devices && st == SVA_OK; d++) {
        for (int s = 0; s < spd && st == SVA_OK; s++)
            st = sva_create(devices[d], &m->ctx[(size_t)d * spd + s]);
        if (st == SVA_OK && (hipSetDevice(devices[d]) != hipSuccess ||
                             hipEventCreateWithFlags(&m->gathered[d], hipEventDisableTiming) !=
                                 hipSuccess))
            st = SVA_ERR_DEVICE;
    }
    if (st == SVA_OK && mode == SVA_MULTI_GATHER_PEER) {
        for (int d = 1; d < n_devices; d++) {
            int can = 0;
            (void)hipSetDevice(devices[d]);
            if (hipDeviceCanAccessPeer(&can, devices[d], devices[0]) == hipSuccess && can) {
                hipError_t e = hipDeviceEnablePeerAccess(devices[0], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) st = SVA_ERR_DEVICE;
                (void)hipGetLastError();
            }
        }
    }
    if (st == SVA_OK && mode == SVA_MULTI_GATHER_RCCL) {
        if (!m->rccl.open(m->last_error)) {
            st = SVA_ERR_UNSUPPORTED;
        } else {
            m->comms.assign(n_devices, nullptr);
            ncclResult_t r = m->rccl.commInitAll(m->comms.data(), n_devices, devices);
            if (r != ncclSuccess) st = SVA_ERR_DEVICE;
        }
    }
    if (st != SVA_OK) {
        sva_multi_destroy(m);
        return st;
    }
    *out = m;
    return SVA_OK;
}

int sva_multi_destroy(void* mp) {
    Multi* m = as_multi(mp);
    if (!m) return SVA_ERR_INVALID_ARG;
    for (size_t i = 0; i < m->ctx.size(); i++)
        if (m->ctx[i]) (void)sva_synchronize(m->ctx[i]);
    for (size_t d = 0; d < m->comms.size(); d++)
        if (m->comms[d]) (void)m->rccl.commDestroy(m->comms[d]);
    for (size_t d = 0; d < m->devices.size(); d++) {
        (void)hipSetDevice(m->devices[d]);
        for (int s = 0; s < m->spd; s++) m->slots[d * m->spd + s].release();
        m->images[d].release();
        if (d < m->copy.size() && m->copy[d]) (void)hipStreamDestroy(m->copy[d]);
        if (d < m->down.size() && m->down[d]) (void)hipStreamDestroy(m->down[d]);
    }
    if (!m->devices.empty()) {
        (void)hipSetDevice(m->devices[0]);
        m->maps0.release();
        m->depth0.release();
        m->nvalid0.release();
    }
    m->stage_in.release();
    m->stage_out.release();
    for (size_t d = 0; d < m->devices.size(); d++) {
        (void)hipSetDevice(m->devices[d]);
        if (d < m->ev_all.size())
            for (hipEvent_t e : m->ev_all[d]) (void)hipEventDestroy(e);
        if (d < m->gathered.size() && m->gathered[d]) (void)hipEventDestroy(m->gathered[d]);
    }
    for (void* c : m->ctx)
        if (c) (void)sva_destroy(c);
    if (m->rccl.lib) dlclose(m->rccl.lib);
    delete m;
    return SVA_OK;
}

int sva_multi_synchronize(void* mp) {
    Multi* m = as_multi(mp);
    if (!m) return SVA_ERR_INVALID_ARG;
    for (void* c : m->ctx) {
        const int s = sva_synchronize(c);
        if (s != SVA_OK) return m->ctx_fail(s, c, "synchronize");
    }
    for (size_t d = 0; d < m->copy.size(); d++) {
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        if (m->copy[d]) MHIP(m, hipStreamSynchronize(m->copy[d]), "synchronize");
        if (m->down[d]) MHIP(m, hipStreamSynchronize(m->down[d]), "synchronize");
    }
    return SVA_OK;
}

const char* sva_multi_last_error(void* mp) {
    Multi* m = as_multi(mp);
    return m ? m->last_error.c_str() : "null engine";
}

int sva_multi_context(void* mp, int d, int s, void** out) {
    Multi* m = as_multi(mp);
    if (!m || !out || d < 0 || d >= m->nd() || s < 0 || s >= m->spd) return SVA_ERR_INVALID_ARG;
    *out = m->ctx[(size_t)d * m->spd + s];
    return SVA_OK;
}

int sva_batch_sgm_d(void* mp, const sva_pair_d* jobs, int n_jobs, int W, int H, size_t pitch,
                    uint16_t* maps, float* sub) {
    Multi* m = as_multi(mp);
    if (!m) return SVA_ERR_INVALID_ARG;
    if (n_jobs < 0 || (n_jobs > 0 && (!jobs || !maps)) || W <= 0 || H <= 0 || pitch < (size_t)W)
        return m->fail(SVA_ERR_INVALID_ARG, "bad batch arguments");
    if (n_jobs == 0) return SVA_OK;
    bool any_sub = false;
    for (int j = 0; j < n_jobs; j++) {
        if (!jobs[j].left || !jobs[j].right || check_params(jobs[j].params))
            return m->fail(SVA_ERR_INVALID_ARG, "bad pair " + std::to_string(j));
        any_sub |= jobs[j].params.subpixel != 0;
    }
    ev_reset(m);
    Plan P;
    make_plan(m->nd(), m->spd, n_jobs, P);
    std::vector<const uint8_t*> l(n_jobs), r(n_jobs);
    std::vector<sva_sgm_params> prm(n_jobs);
    std::vector<std::vector<hipEvent_t>> none(n_jobs);
    for (int j = 0; j < n_jobs; j++) {
        l[j] = jobs[j].left;
        r[j] = jobs[j].right;
        prm[j] = jobs[j].params;
    }
    return run_pairs(m, P, l, r, prm, none, W, H, pitch, maps, any_sub ? sub : nullptr);
}

int sva_array_depth(void* mp, const uint8_t* const* images, int n_images, int W, int H,
                    size_t pitch, const sva_array_pair* pairs, int n_pairs,
                    const int32_t* group_start, int n_groups, double f, double pixel_size,
                    double* depth, uint8_t* n_valid, uint16_t* maps) {
    Multi* m = as_multi(mp);
    if (!m) return SVA_ERR_INVALID_ARG;
    if (!images || n_images <= 0 || !pairs || n_pairs <= 0 || !group_start || n_groups <= 0 ||
        !depth || W <= 0 || H <= 0 || pitch < (size_t)W)
        return m->fail(SVA_ERR_INVALID_ARG, "bad array arguments");
    if (group_start[0] != 0 || group_start[n_groups] != n_pairs)
        return m->fail(SVA_ERR_INVALID_ARG, "group_start must run from 0 to n_pairs");
    for (int g = 0; g < n_groups; g++) {
        const int n = group_start[g + 1] - group_start[g];
        if (n <= 0 || n > 32) return m->fail(SVA_ERR_UNSUPPORTED, "groups of 1..32 pairs");
        // the fusion rejects one `invalid` value per group
        for (int j = group_start[g] + 1; j < group_start[g + 1]; j++)
            if (pairs[j].params.invalid != pairs[group_start[g]].params.invalid)
                return m->fail(SVA_ERR_INVALID_ARG,
                               "params.invalid differs within group " + std::to_string(g));
    }
    for (int j = 0; j < n_pairs; j++) {
        const sva_array_pair& q = pairs[j];
        if (q.ref < 0 || q.ref >= n_images || q.other < 0 || q.other >= n_images ||
            !images[q.ref] || !images[q.other] || check_params(q.params))
            return m->fail(SVA_ERR_INVALID_ARG, "bad pair " + std::to_string(j));
    }
    ev_reset(m);
    const size_t np = (size_t)W * H;
    Plan P;
    make_plan(m->nd(), m->spd, n_pairs, P);
    if (m->copy.empty()) {
        m->copy.assign(m->nd(), nullptr);
        m->down.assign(m->nd(), nullptr);
        for (int d = 0; d < m->nd(); d++) {
            MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
            MHIP(m, hipStreamCreateWithFlags(&m->copy[d], hipStreamNonBlocking), "stream");
            MHIP(m, hipStreamCreateWithFlags(&m->down[d], hipStreamNonBlocking), "stream");
        }
    }
    // 1. which views each device needs, staged once into pinned memory
    std::vector<std::vector<int>> slot_of(m->nd(), std::vector<int>(n_images, -1));
    std::vector<int> n_need(m->nd(), 0);
    std::vector<char> used(n_images, 0);
    for (int j = 0; j < n_pairs; j++)
        for (int v : {pairs[j].ref, pairs[j].other}) {
            used[v] = 1;
            int& s = slot_of[P.dev[j]][v];
            if (s < 0) s = n_need[P.dev[j]]++;
        }
    std::vector<int> pin_slot(n_images, -1);
    int n_pin = 0;
    for (int v = 0; v < n_images; v++)
        if (used[v]) pin_slot[v] = n_pin++;
    // the previous call's uploads must be done before the pinned staging is rewritten
    for (int d = 0; d < m->nd(); d++) {
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        MHIP(m, hipStreamSynchronize(m->copy[d]), "synchronize");
    }
    MHIP(m, m->stage_in.ensure((size_t)n_pin * np), "pinned staging");
    // 2. uploads on each device's copy stream, one event per (device, view);
    // the images buffer is reused only after the previous call's pairs ran
    std::vector<std::vector<hipEvent_t>> up_ev(m->nd(), std::vector<hipEvent_t>(n_images));
    for (int v = 0; v < n_images; v++)
        if (used[v])
            copy_plane((uint8_t*)m->stage_in.ptr + (size_t)pin_slot[v] * np, images[v], W, H, pitch);
    for (int d = 0; d < m->nd(); d++) {
        if (!n_need[d]) continue;
        MHIP(m, hipSetDevice(m->devices[d]), "hipSetDevice");
        for (int s = 0; s < m->spd; s++) {
            int st = stream_after(m, d, m->st(d, s), m->copy[d]);
            if (st) return st;
        }
        MHIP(m, m->images[d].ensure((size_t)n_need[d] * np), "view workspace");
        for (int v = 0; v < n_images; v++) {
            if (slot_of[d][v] < 0) continue;
            MHIP(m, hipMemcpyAsync((uint8_t*)m->images[d].ptr + (size_t)slot_of[d][v] * np,
                                   (uint8_t*)m->stage_in.ptr + (size_t)pin_slot[v] * np, np,
                                   hipMemcpyHostToDevice, m->copy[d]),
                 "upload");
            MHIP(m, ev_on(m, d, &up_ev[d][v]), "event");
            MHIP(m, hipEventRecord(up_ev[d][v], m->copy[d]), "event record");
        }
    }
    // 3. pairs + gather into maps0 on device 0
    MHIP(m, hipSetDevice(m->devices[0]), "hipSetDevice");
    MHIP(m, hipStreamSynchronize(m->st(0, 0)), "synchronize");   // maps0/depth0 reuse
    MHIP(m, m->maps0.ensure(np * 2 * n_pairs), "map workspace");
    MHIP(m, m->depth0.ensure(np * 8 * n_groups), "depth workspace");
    MHIP(m, m->nvalid0.ensure(np * n_groups), "depth workspace");
    std::vector<const uint8_t*> l(n_pairs), r(n_pairs);
    std::vector<sva_sgm_params> prm(n_pairs);
    std::vector<std::vector<hipEvent_t>> waits(n_pairs);
    for (int j = 0; j < n_pairs; j++) {
        const int d = P.dev[j];
        const uint8_t* base = (const uint8_t*)m->images[d].ptr;
        l[j] = base + (size_t)slot_of[d][pairs[j].ref] * np;
        r[j] = base + (size_t)slot_of[d][pairs[j].other] * np;
        prm[j] = pairs[j].params;
        prm[j].subpixel = 0;
        waits[j] = {up_ev[d][pairs[j].ref], up_ev[d][pairs[j].other]};
    }
    uint16_t* maps0 = (uint16_t*)m->maps0.ptr;
    int st = run_pairs(m, P, l, r, prm, waits, W, H, W, maps0, nullptr);
    if (st) return st;
    // 4. fusion per group on device 0, each group's download as soon as it is fused
    MHIP(m, hipSetDevice(m->devices[0]), "hipSetDevice");
    MHIP(m, m->stage_out.ensure(np * (8 + (n_valid ? 1 : 0)) * n_groups +
                                (maps ? np * 2 * n_pairs : 0)),
         "pinned staging");
    uint8_t* pout = (uint8_t*)m->stage_out.ptr;
    double* depth0 = (double*)m->depth0.ptr;
    uint8_t* nv0 = (uint8_t*)m->nvalid0.ptr;
    std::vector<double> bases(n_pairs);
    for (int j = 0; j < n_pairs; j++) bases[j] = pairs[j].baseline;
    for (int g = 0; g < n_groups; g++) {
        const int j0 = group_start[g], n = group_start[g + 1] - j0;
        st = sva_fuse_depth_d(m->ctx[0], maps0 + (size_t)j0 * np, n, W, H, &bases[j0], f,
                              pixel_size, pairs[j0].params.invalid, depth0 + (size_t)g * np,
                              nv0 + (size_t)g * np);
        if (st) return m->ctx_fail(st, m->ctx[0], "fuse");
        if ((st = stream_after(m, 0, m->st(0, 0), m->down[0]))) return st;
        MHIP(m, hipMemcpyAsync(pout + (size_t)g * np * 8, depth0 + (size_t)g * np, np * 8,
                               hipMemcpyDeviceToHost, m->down[0]),
             "download");
        if (n_valid)
            MHIP(m, hipMemcpyAsync(pout + (size_t)n_groups * np * 8 + (size_t)g * np,
                                   nv0 + (size_t)g * np, np, hipMemcpyDeviceToHost, m->down[0]),
                 "download");
    }
    if (maps)
        MHIP(m, hipMemcpyAsync(pout + np * (8 + (n_valid ? 1 : 0)) * n_groups, maps0,
                               np * 2 * n_pairs, hipMemcpyDeviceToHost, m->down[0]),
             "download");
    MHIP(m, hipStreamSynchronize(m->down[0]), "synchronize");
    std::memcpy(depth, pout, np * 8 * n_groups);
    if (n_valid) std::memcpy(n_valid, pout + (size_t)n_groups * np * 8, np * n_groups);
    if (maps) std::memcpy(maps, pout + np * (8 + (n_valid ? 1 : 0)) * n_groups, np * 2 * n_pairs);
    return SVA_OK;
}

}  // extern "C"
