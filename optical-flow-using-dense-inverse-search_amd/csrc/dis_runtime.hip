// dis_runtime.hip -- the C-ABI (include/dis_abi.h): parameter validation,
// geometry, device workspace and the per-batch launch sequence.
//
// The launch sequence is the reference's control flow restated for a batch of
// pairs resident in HBM: src/main.cpp:135-198 (pad/convert, pyramid, upsample,
// crop) around src/optical_flow.cpp:67-91 (coarse-to-fine scale loop).
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>

#include "dis_kernels.h"
#include "dis_plan.h"

namespace {


thread_local std::string g_err;

dis_status fail(dis_status s, const std::string& msg)
{
    g_err = msg;
    return s;
}

#define DIS_HIP(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(DIS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    } while (0)

}  // namespace

namespace dis {

// error reporting for the host-only translation units (dis_io.cpp)
dis_status set_error(dis_status s, const std::string& msg) { return fail(s, msg); }

bool make_geometry(const dis_params& p, int W, int H, Geometry* g)
{
    std::memset(g, 0, sizeof(*g));
    g->W = W;
    g->H = H;
    g->C = p.coarsest_scale;
    g->F = p.finest_scale;
    g->ps = p.patch_size;
    g->iters = p.iterations;
    g->norm = p.patch_normalization ? 1 : 0;
    // src/main.cpp:139-155
    const int sf = 1 << g->C;
    const int padw = (W % sf) ? sf - W % sf : 0;
    const int padh = (H % sf) ? sf - H % sf : 0;
    g->Wp = W + padw;
    g->Hp = H + padh;
    g->pad_left = padw / 2;
    g->pad_top = padh / 2;
    // src/optical_flow.cpp:38
    const int st = (int)std::floor((float)p.patch_size * (1.0f - p.patch_overlap));
    g->steps = st < 1 ? 1 : st;
    long long poff = 0, uoff = 0, doff = 0;
    for (int l = 0; l <= g->C; ++l) {
        LevelGeom& L = g->lv[l];
        const float sc = std::pow(2.0f, (float)-l);  // src/optical_flow.cpp:50-53
        L.W = (int)((float)g->Wp * sc);
        L.H = (int)((float)g->Hp * sc);
        if (L.W < 1 || L.H < 1) return false;
        L.steps = g->steps;
        // src/patch_grid.cpp:20-23
        L.npw = (int)std::ceil((float)L.W / (float)g->steps);
        L.nph = (int)std::ceil((float)L.H / (float)g->steps);
        L.offw = (L.W - (L.npw - 1) * g->steps) / 2;
        L.offh = (L.H - (L.nph - 1) * g->steps) / 2;
        L.n = L.npw * L.nph;
        // src/optical_flow.cpp:55-57
        L.tmp_lb = -(float)p.patch_size / 2;
        L.tmp_ub_w = (float)(L.W + p.patch_size / 2 - 2);
        L.tmp_ub_h = (float)(L.H + p.patch_size / 2 - 2);
        L.plane_off = poff;
        L.u_off = uoff;
        L.dense_off = doff;
        poff += (long long)L.W * L.H;
        uoff += L.n;
        doff += (long long)L.W * L.H;
    }
    g->plane_stride = (poff + 63) & ~63LL;
    g->u_stride = (uoff + 31) & ~31LL;
    g->dense_stride = (doff + 31) & ~31LL;
    return true;
}

}  // namespace dis

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
// level patches x pairs up to which 8 lanes per patch is used (A/B: 65536
// -2.6 %); above it 2 lanes per patch (LPP 1 / 4 measured slower)
constexpr long long kLpp8MaxPatches = 16384;

// Lanes per patch for the patch_size-8 search at one level. Few patches leave
// the chip idle and the level is bound by one wave's serial iteration chain:
// spend more lanes per patch (shorter chain). Many patches make it VALU-bound:
// 2 lanes per patch does the least total work.
static int search8_lanes(int variant, long long patches, int steps)
{
    if (variant == 2) return 4;
    if (variant == 3 || variant == 9) return 2;
    if (variant == 4) return 8;
    if (variant == 5) return dis::search8_lpp1_fits(steps) ? 1 : 2;
    if (variant == 6) return 64;  // one wave per patch (exact, non-paper levels)
    return patches <= kLpp8MaxPatches ? 8 : 2;
}

// per sub-batch: the levels' fallback list counts (k_search8_fb)
constexpr size_t kFbCounters = dis::kMaxLevels;

// Host-frame path state (dis_calc_batch_u8 with DIS_MEM_HOST), made on the
// first host call: the batch runs in chunks of `chunk` pairs through two
// device staging slots, so that the upload of chunk j+1, the computation of
// chunk j and the download of chunk j-1 overlap (the reference's own pattern
// is host frames in, host flow out per pair, src/main.cpp:115-116,184-189).
// The copies go straight between the caller's buffers and the device: a
// hipMemcpyAsync on pageable memory runs at the DMA rate but returns only when
// it is done (tools/host_xfer_probe.hip), so the downloads are issued by a
// thread of their own while the calling thread uploads and enqueues. Staging
// through page-locked buffers with threaded host copies, and host waits
// instead of stream waits in front of the copies, measured slower (DESIGN.md
// 4, host-frame path).
struct HostPipe {
    int chunk = 0;
    size_t frame = 0;                 // bytes of one frame (W * H)
    uint8_t* din[2] = {};             // device: chunk I0 frames, then chunk I1 frames
    float2* dout[2] = {};             // device: chunk flows
    hipStream_t up = nullptr, down = nullptr;
    hipEvent_t up_done[2] = {}, comp_done[2] = {}, down_done[2] = {};
    bool comp_pending[2] = {}, down_pending[2] = {};
    // the download thread: jobs in chunk order; `issued` counts the jobs whose
    // copy has been issued and whose down_done event has been recorded
    struct Job {
        char* dst;
        const char* src;
        size_t bytes;
        int slot;
    };
    std::thread th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<Job> q;
    long long posted = 0, issued = 0;
    hipError_t err = hipSuccess;
    bool stop = false;
    int device = 0;
    // what the last host call did (dis_host_pipeline_info)
    int last_chunks = 0, last_direct_in = 0, last_direct_out = 0;

    void run()
    {
        (void)hipSetDevice(device);
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                j = q.front();
                q.erase(q.begin());
            }
            hipError_t e = hipStreamWaitEvent(down, comp_done[j.slot], 0);
            if (e == hipSuccess) e = hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost, down);
            if (e == hipSuccess) e = hipEventRecord(down_done[j.slot], down);
            std::lock_guard<std::mutex> l(mu);
            if (e != hipSuccess && err == hipSuccess) err = e;
            ++issued;
            done_cv.notify_all();
        }
    }
    void post(const Job& j)
    {
        {
            std::lock_guard<std::mutex> l(mu);
            q.push_back(j);
            ++posted;
        }
        cv.notify_one();
    }
    // wait until the first `k` posted jobs are issued; the first error seen
    hipError_t wait_issued(long long k)
    {
        std::unique_lock<std::mutex> l(mu);
        done_cv.wait(l, [&] { return issued >= k; });
        const hipError_t e = err;
        err = hipSuccess;
        return e;
    }
    ~HostPipe()
    {
        if (th.joinable()) {
            {
                std::lock_guard<std::mutex> l(mu);
                stop = true;
            }
            cv.notify_all();
            th.join();
        }
        // copies of a call that failed part-way may still be in flight
        if (up) (void)hipStreamSynchronize(up);
        if (down) (void)hipStreamSynchronize(down);
        for (int s = 0; s < 2; ++s) {
            hipFree(din[s]);
            hipFree(dout[s]);
            for (hipEvent_t e : {up_done[s], comp_done[s], down_done[s]})
                if (e) hipEventDestroy(e);
        }
        if (up) hipStreamDestroy(up);
        if (down) hipStreamDestroy(down);
    }
};

struct dis_ctx {
    dis_params p;
    dis::Geometry g;
    int device = 0;
    int max_batch = 1;
    int debug = 0;
    int variant = 0;  // 0 auto, 1 generic only, 2/3/4/5/6: patch_size-8 search with 4/2/8/1/64 lanes per patch
    int last_batch = 0;
    int last_nsub = 1;  // sub-batches of the last calc (their fallback counters, DIS_STAGE_FALLBACK)
    hipStream_t own = nullptr;
    static constexpr int kMaxSub = 8;
    int nsub = 2;                        // sub-batch streams per calc (dis_set_concurrency)
    int precision = 0;                   // dis_set_precision: DIS_PRECISION_EXACT / _FMA
    hipStream_t sub[kMaxSub] = {};
    hipEvent_t fork = nullptr;
    // end of the previous call's work on its stream: every call first orders
    // its stream after it, so calls on different streams (calc_device on a
    // caller stream, then calc_batch on `own`) never overlap on the workspace
    hipEvent_t done = nullptr;
    bool done_pending = false;
    hipStream_t done_stream = nullptr;  // the stream `done` was recorded on
    // the next call must wait for `done` unless it is on that same stream
    // (stream order already serialises it; skipping the wait packet saves the
    // inter-call gap)
    bool needs_wait(hipStream_t s) const { return done_pending && s != done_stream; }
    hipEvent_t join[kMaxSub] = {};
    // variational refinement: its ~16 launches per fixed-point iteration per level
    // are replayed as one HIP graph per (sub-batch, level), captured on first use
    // (all pointers are context workspace; re-captured when the slice changes)
    struct VrGraph {
        hipGraphExec_t exec = nullptr;
        int n = -1, p0 = -1;
    } vrg[kMaxSub][dis::kMaxLevels];
    hipStream_t cap = nullptr;  // capture-only stream
    // The whole batch call (both sub-batches' pyramid, level searches and
    // output, with the fork/join) replayed as one HIP graph: dis_set_graphs,
    // default on. A small LRU of executable graphs keyed by the call (buffers,
    // batch size, sub-batches, precision, variant): a caller that ping-pongs
    // a few buffer sets replays without re-capturing. A miss re-captures into
    // the least recently used slot and updates its exec in place -- only after
    // that exec's last replay has finished (`last`): the update rewrites the
    // kernel arguments an unstarted node of that replay would still read.
    int graphs = 1;
    static constexpr int kGraphCache = 4;
    struct MainGraph {
        hipGraphExec_t exec = nullptr;
        hipEvent_t last = nullptr;  // recorded after this exec's latest launch
        bool launched = false;
        unsigned long long used = 0;  // LRU clock
        int n = -1, nsub = -1, precision = -1, variant = -1;
        int subs = 1;  // sub-batches the captured call ran (last_nsub on replay)
        const void *i0 = nullptr, *i1 = nullptr;
        void* flow = nullptr;
        size_t stride = 0, pair_stride = 0;
    } mg[kGraphCache];
    unsigned long long graph_clock = 0;
    // workspace (device)
    float* img0 = nullptr;
    float* img1 = nullptr;
    float* dx = nullptr;
    float* dy = nullptr;
    float2* pu = nullptr;
    float2* dense = nullptr;
    float* vr_ws = nullptr;  // variational refinement workspace (kVarRefPlanes planes per pair)
    long long vr_plane = 0;
    // patch-search fallback lists (dis_search8.hip k_search8_fb): per sub-batch
    // k, kFbCounters list counts (one per level) at fb + k * kFbCounters, then
    // per (k, level) a list of up to blocks(level) * pairs entries at
    // fb + fb_list_off[k][level]
    int* fb = nullptr;
    size_t fb_list_off[8][dis::kMaxLevels] = {};
    // host-frame path (DIS_MEM_HOST): device slots, streams and the download
    // thread made on the first host call; dis_set_host_pipeline sets the chunk
    // (0 = auto)
    std::unique_ptr<HostPipe> hp;
    int host_chunk = 0;
    // kernel timing
    int timing = 0;
    struct Rec {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<hipEvent_t> pool;
    std::vector<Rec> recs;
    size_t pool_next = 0;
    static constexpr int kKinds = 6;  // dis_kernel_time classes
    int launches[kKinds] = {};
    double total_ms[kKinds] = {};
    long long dropped = 0;  // records lost to a failed event creation (dis_kernel_time fails then)
};

namespace {

dis_status check_params(const dis_params* p, int W, int H)
{
    if (!p) return fail(DIS_ERR_INVALID_ARGUMENT, "params is null");
    if (W < 1 || H < 1) return fail(DIS_ERR_INVALID_ARGUMENT, "width and height must be >= 1");
    if ((long long)W * H > (1LL << 28)) return fail(DIS_ERR_INVALID_ARGUMENT, "frame too large");
    if (p->patch_size < 2 || p->patch_size > 16 || (p->patch_size & 1))
        return fail(DIS_ERR_INVALID_ARGUMENT,
                    "patch_size must be even and in [2,16] (odd sizes are broken in the reference, Q11)");
    if (!(p->patch_overlap >= 0.0f && p->patch_overlap < 1.0f))
        return fail(DIS_ERR_INVALID_ARGUMENT, "patch_overlap must be in [0,1)");
    if (p->finest_scale < 0 || p->coarsest_scale < p->finest_scale)
        return fail(DIS_ERR_INVALID_ARGUMENT, "need 0 <= finest_scale <= coarsest_scale");
    if (p->coarsest_scale >= dis::kMaxLevels - 1)
        return fail(DIS_ERR_INVALID_ARGUMENT, "coarsest_scale too large");
    if (p->iterations < 0) return fail(DIS_ERR_INVALID_ARGUMENT, "iterations must be >= 0");
    if (p->var_refine_iters < 0 || p->var_refine_iters > 64)
        return fail(DIS_ERR_INVALID_ARGUMENT, "var_refine_iters must be in [0, 64]");
    if (p->paper_mode != 0 && p->paper_mode != 1) return fail(DIS_ERR_INVALID_ARGUMENT, "paper_mode must be 0 or 1");
    const int sf = 1 << p->coarsest_scale;
    const int Wp = W + ((W % sf) ? sf - W % sf : 0), Hp = H + ((H % sf) ? sf - H % sf : 0);
    if ((Wp >> p->coarsest_scale) < 1 || (Hp >> p->coarsest_scale) < 1)
        return fail(DIS_ERR_INVALID_ARGUMENT, "frame smaller than 2^coarsest_scale");
    return DIS_OK;
}

void free_ws(dis_ctx* c)
{
    hipFree(c->img0);
    hipFree(c->img1);
    hipFree(c->dx);
    hipFree(c->dy);
    hipFree(c->pu);
    hipFree(c->dense);
    hipFree(c->fb);
    c->fb = nullptr;
    hipFree(c->vr_ws);
    c->vr_ws = nullptr;
    c->hp.reset();
    c->img0 = c->img1 = c->dx = c->dy = nullptr;
    c->pu = c->dense = nullptr;
}

// Per-launch timing: when enabled, hands out an event pair from the pool to be
// attached to the next dispatch (hipExtLaunchKernelGGL) and books it under
// `kind` (and `kind2` if >= 0).
dis::Timing timing(dis_ctx* c, int kind, int kind2 = -1)
{
    dis::Timing t;
    if (!c->timing) return t;
    if (c->pool_next + 2 > c->pool.size()) {  // grow: a record is never dropped
        const size_t n0 = c->pool.size();
        c->pool.resize(n0 + 1024);
        for (size_t i = n0; i < c->pool.size(); ++i)
            if (hipEventCreate(&c->pool[i]) != hipSuccess) {
                c->pool.resize(i);
                c->dropped += 1;
                return t;
            }
    }
    t.start = c->pool[c->pool_next++];
    t.stop = c->pool[c->pool_next++];
    c->recs.push_back({kind, t.start, t.stop});
    if (kind2 >= 0) c->recs.push_back({kind2, t.start, t.stop});
    return t;
}

// Largest float s with sqrtf(s) <= thr (sqrtf is correctly rounded and
// monotone, so `sqrtf(s) > thr` <=> `s > thr_sq`; src/patch.cpp:185).
float sqrt_threshold(float thr)
{
    float s = thr * thr;
    while (std::sqrt(s) > thr) s = std::nextafter(s, 0.0f);
    while (std::sqrt(std::nextafter(s, INFINITY)) <= thr) s = std::nextafter(s, INFINITY);
    return s;
}

// cv::resize HResizeLinear: first destination column whose source index
// reaches wF-1; columns from there on take S[wF-1] alone (src/main.cpp:195).
int upsample_xmax(const dis::Geometry& g)
{
    const int wF = g.lv[g.F].W;
    const double inv = 1.0 / (double)std::pow(2.0f, (float)g.F);
    for (int d = 0; d < g.Wp; ++d) {
        const float fx = (float)((d + 0.5) * inv - 0.5);
        int sx = (int)std::floor(fx);
        if (sx < 0) sx = 0;
        if (sx + 1 >= wF) return d;
    }
    return g.Wp;
}

constexpr int kStageFront = 1000, kStageBack = -1000;  // other stages: the level index

// roctx markers, resolved at first use with dlopen (no link-time dependency:
// without the roctx library, or without a tool attached, they are no-ops).
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx()
    {
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};
const Roctx& roctx()
{
    static const Roctx r;
    return r;
}

// roctx range around the host-side enqueue of one stage of one sub-batch
// ("dis: level 3 sub 1"), or of a call phase: visible in rocprofv3
// --marker-trace timelines.
struct StageRange {
    StageRange(int stage, int sub)
    {
        char b[48];
        if (stage == kStageFront)
            std::snprintf(b, sizeof b, "dis: pyramid sub %d", sub);
        else if (stage == kStageBack)
            std::snprintf(b, sizeof b, "dis: output sub %d", sub);
        else
            std::snprintf(b, sizeof b, "dis: level %d sub %d", stage, sub);
        if (roctx().push) roctx().push(b);
    }
    explicit StageRange(const char* what)
    {
        if (roctx().push) roctx().push(what);
    }
    ~StageRange()
    {
        if (roctx().pop) roctx().pop();
    }
    StageRange(const StageRange&) = delete;
    StageRange& operator=(const StageRange&) = delete;
};

// One mutex per device guards the device's pooled sub-batch streams
// (sub_streams): held across a context's eager enqueue of a forked batch call
// and across a graph capture (which puts the pooled streams into capture
// mode), so concurrent contexts on different host threads never interleave
// work on a shared stream while it is being captured.
std::mutex& pool_mutex(int device)
{
    static std::mutex mu;
    static std::map<int, std::mutex> per_device;
    std::lock_guard<std::mutex> lock(mu);
    return per_device[device];
}

// k_densify arguments for level l of a sub-batch's workspace slice
dis::DensifyArgs densify_args(const dis_ctx* c, int l, const float* img0, const float* img1, float2* pu,
                              float2* dense)
{
    const dis::Geometry& g = c->g;
    const dis::LevelGeom& L = g.lv[l];
    dis::DensifyArgs d{};
    d.img0 = img0 + L.plane_off;
    d.img1 = img1 + L.plane_off;
    d.plane_stride = g.plane_stride;
    d.paper = c->p.paper_mode != 0 ? 1 : 0;
    d.u = pu + L.u_off;
    d.dense = dense + L.dense_off;
    d.u_stride = g.u_stride;
    d.dense_stride = g.dense_stride;
    d.W = L.W;
    d.H = L.H;
    d.ps = g.ps;
    d.steps = L.steps;
    d.npw = L.npw;
    d.nph = L.nph;
    d.offw = L.offw;
    d.offh = L.offh;
    return d;
}

// One stage of the path for n pairs already resident in device memory: the
// front end (pyramid), one level (search, and densify + refinement when on),
// or the back end (output). run_batches issues the stages stage-major across
// the sub-batches, so every sub-batch's next kernels are queued early even
// when the host is slow to enqueue a long stage.
dis_status run_batch(dis_ctx* c, int sub, int n, int p0, const uint8_t* I0, const uint8_t* I1, size_t stride,
                     size_t pair_stride, float2* flow, hipStream_t s, int stage)
{
    // this sub-batch's fallback counts (one per level)
    int* const fb_count = c->fb + (size_t)sub * kFbCounters;
    const dis::Geometry& g = c->g;
    // this sub-batch's slice of the workspace (pairs p0 .. p0+n-1)
    float* const img0 = c->img0 + (size_t)p0 * g.plane_stride;
    float* const img1 = c->img1 + (size_t)p0 * g.plane_stride;
    float* const gdx = c->dx + (size_t)p0 * g.plane_stride;
    float* const gdy = c->dy + (size_t)p0 * g.plane_stride;
    float2* const pu = c->pu + (size_t)p0 * g.u_stride;
    float2* const dense = c->dense + (size_t)p0 * g.dense_stride;
    const bool fast = g.ps == 8 && c->variant != 1;
    const bool vr = c->p.var_refine_iters > 0;
    const bool paper = c->p.paper_mode != 0;
    if (stage == kStageFront) {
        if (fast && g.C >= 1) {
            dis::PyramidArgs pa{};
            pa.I0 = I0;
            pa.I1 = I1;
            pa.stride = stride;
            pa.pair_stride = pair_stride;
            pa.W = g.W;
            pa.H = g.H;
            pa.Wp = g.Wp;
            pa.Hp = g.Hp;
            pa.pl = g.pad_left;
            pa.pt = g.pad_top;
            pa.img0 = img0;
            pa.img1 = img1;
            pa.plane_stride = g.plane_stride;
            pa.levels = std::min(g.C, 6);
            pa.write_l0 = (g.F == 0 || c->debug) ? 1 : 0;
            pa.zero = fb_count;
            pa.nzero = g.C + 1;
            pa.dword_ok = ((reinterpret_cast<uintptr_t>(I0) | reinterpret_cast<uintptr_t>(I1) | stride |
                            (n > 1 ? pair_stride : 0) | (size_t)g.pad_left) & 3) == 0;
            pa.qword_ok = ((reinterpret_cast<uintptr_t>(I0) | reinterpret_cast<uintptr_t>(I1) | stride |
                            (n > 1 ? pair_stride : 0) | (size_t)g.pad_left) & 15) == 0;
            for (int l = 0; l <= g.C; ++l) {
                pa.off[l] = g.lv[l].plane_off;
                pa.w[l] = g.lv[l].W;
            }
            if (dis::pyramid2_fits(pa))  // the two-kernel streaming pyramid (dis_pyramid.hip)
                DIS_HIP(dis::launch_pyramid2(pa, n, s, timing(c, 0)));
            else
                DIS_HIP(dis::launch_pyramid(pa, n, s, timing(c, 0)));
            for (int l = pa.levels + 1; l <= g.C; ++l) DIS_HIP(dis::launch_down2(g, l, img0, img1, n, s));
        } else {
            // (zeroed on every path: DIS_STAGE_FALLBACK reports them after any calc)
            DIS_HIP(hipMemsetAsync(fb_count, 0, sizeof(int) * (g.C + 1), s));
            DIS_HIP(dis::launch_level0(I0, I1, stride, pair_stride, g, img0, img1, n, s));
            for (int l = 1; l <= g.C; ++l) DIS_HIP(dis::launch_down2(g, l, img0, img1, n, s));
        }
        if (!fast || c->debug)  // the fast search computes its template gradients itself
            for (int l = g.F; l <= g.C; ++l) DIS_HIP(dis::launch_sobel(g, l, img0, gdx, gdy, n, s));
    }
    // the fast search's arguments for level lq of this sub-batch
    auto make_s8 = [&](int lq) {
        const dis::LevelGeom& Lq = g.lv[lq];
        dis::Search8Args b{};
        b.img0 = img0;
        b.img1 = img1;
        b.u_coarse = (lq < g.C) ? pu + g.lv[lq + 1].u_off : nullptr;
        b.u_out = pu + Lq.u_off;
        b.plane_stride = g.plane_stride;
        b.plane_off = Lq.plane_off;
        b.u_stride = g.u_stride;
        b.W = Lq.W;
        b.H = Lq.H;
        b.steps = Lq.steps;
        b.npw = Lq.npw;
        b.nph = Lq.nph;
        b.offw = Lq.offw;
        b.offh = Lq.offh;
        if (lq < g.C) {
            b.c_npw = g.lv[lq + 1].npw;
            b.c_nph = g.lv[lq + 1].nph;
            b.c_offw = g.lv[lq + 1].offw;
            b.c_offh = g.lv[lq + 1].offh;
        }
        b.tmp_lb = Lq.tmp_lb;
        b.tmp_ub_w = Lq.tmp_ub_w;
        b.tmp_ub_h = Lq.tmp_ub_h;
        b.thr_sq = sqrt_threshold((float)g.ps / 2);
        b.lanes_per_patch = search8_lanes(c->variant, (long long)Lq.npw * Lq.nph * n, Lq.steps);
        b.tile_stride = dis::search8_tile_stride(Lq.steps, b.lanes_per_patch);
        b.quad = dis::search8_tile_quad(Lq.steps, b.lanes_per_patch);
        b.tile_cap = c->variant == 9 ? 24 : 0;  // variant 9: most blocks through the fallback list
        b.fb_count = fb_count + lq;
        b.fb_list = c->fb + c->fb_list_off[sub][lq];
        b.paper = paper ? 1 : 0;
        b.iters = g.iters;
        b.norm = g.norm;
        b.fma = (c->precision == DIS_PRECISION_FMA && !paper) ? 1 : 0;
        return b;
    };
    for (int l = g.C; l >= g.F; --l) {  // src/optical_flow.cpp:67-91
        if (l != stage) continue;
        const dis::LevelGeom& L = g.lv[l];
        dis::SearchArgs a{};
        a.img0 = img0;
        a.img1 = img1;
        a.dx = gdx;
        a.dy = gdy;
        a.dense_coarse = (l < g.C) ? dense + g.lv[l + 1].dense_off : nullptr;
        a.u_out = pu + L.u_off;
        a.plane_stride = g.plane_stride;
        a.plane_off = L.plane_off;
        a.dense_stride = g.dense_stride;
        a.u_stride = g.u_stride;
        a.phys_pad = 0;
        a.W = L.W;
        a.H = L.H;
        a.steps = L.steps;
        a.npw = L.npw;
        a.nph = L.nph;
        a.offw = L.offw;
        a.offh = L.offh;
        a.n = L.n;
        a.tmp_lb = L.tmp_lb;
        a.tmp_ub_w = L.tmp_ub_w;
        a.tmp_ub_h = L.tmp_ub_h;
        a.outlier = (float)g.ps / 2;
        a.iters = g.iters;
        a.norm = g.norm;
        a.paper = paper ? 1 : 0;
        if (fast) {
            dis::Search8Args b = make_s8(l);
            if (paper && l < g.C) {  // the weighted coarse-to-fine init reads the coarser level's planes
                b.c_plane_off = g.lv[l + 1].plane_off;
                b.c_W = g.lv[l + 1].W;
                b.c_H = g.lv[l + 1].H;
            }
            if (vr && l < g.C) {  // refined dense flows: init from the coarser level's dense field
                b.dense_coarse = dense + g.lv[l + 1].dense_off;
                b.dense_stride = g.dense_stride;
            }
            if (b.lanes_per_patch == 64 && (paper || b.fma)) {  // exact, non-paper only
                b.lanes_per_patch = 2;
                b.tile_stride = dis::search8_tile_stride(L.steps, 2);
                b.quad = dis::search8_tile_quad(L.steps, 2);
            }
            DIS_HIP(dis::launch_search8(b, n, s, timing(c, 1, l == g.F ? 2 : -1)));
        } else {
            DIS_HIP(dis::launch_search_generic(a, g.ps, n, s, timing(c, 1, l == g.F ? 2 : -1)));
        }
        // the fast path materialises dense fields only under refinement (the next
        // level initialises from the refined field); otherwise the search fuses
        // the coarser level's densification at its sampled pixels and the output
        // kernel densifies the finest level
        if (fast && !c->debug && !vr) continue;
        DIS_HIP(dis::launch_densify(densify_args(c, l, img0, img1, pu, dense), n, s));
        if (vr) {  // variational refinement of the level's dense flow
            dis::VarRefArgs v{};
            v.img0 = img0 + L.plane_off;
            v.img1 = img1 + L.plane_off;
            v.plane_stride = g.plane_stride;
            v.flow = dense + L.dense_off;
            v.flow_stride = g.dense_stride;
            v.ws = c->vr_ws + (size_t)p0 * dis::kVarRefPlanes * c->vr_plane;
            v.ws_plane = c->vr_plane;
            v.ws_stride = dis::kVarRefPlanes * c->vr_plane;
            v.W = L.W;
            v.H = L.H;
            v.iters = c->p.var_refine_iters;
            if (c->timing) {  // eager, events around the finest level's refinement launches
                auto tf = [](void* cc, int kind) { return timing(static_cast<dis_ctx*>(cc), 4 + kind); };
                DIS_HIP(dis::launch_var_refine(v, n, s, l == g.F ? +tf : nullptr, c));
                continue;
            }
            auto& G = c->vrg[sub][l];  // the level's launches replayed as one HIP graph
            if (G.n != n || G.p0 != p0) {
                if (G.exec) hipGraphExecDestroy(G.exec);
                G.exec = nullptr;
                G.n = G.p0 = -1;
                hipGraph_t graph = nullptr;
                DIS_HIP(hipStreamBeginCapture(c->cap, hipStreamCaptureModeThreadLocal));
                const hipError_t e = dis::launch_var_refine(v, n, c->cap);
                const hipError_t e2 = hipStreamEndCapture(c->cap, &graph);
                DIS_HIP(e);
                DIS_HIP(e2);
                const hipError_t e3 = hipGraphInstantiate(&G.exec, graph, nullptr, nullptr, 0);
                hipGraphDestroy(graph);
                DIS_HIP(e3);
                G.n = n;
                G.p0 = p0;
            }
            DIS_HIP(hipGraphLaunch(G.exec, s));
        }
    }
    if (stage != kStageBack) return DIS_OK;
    dis::OutputArgs o{};
    bool fused_out = false;
    if (fast) {
        const dis::LevelGeom& LF = g.lv[g.F];
        o.u = pu + LF.u_off;
        o.flow = flow;
        o.u_stride = g.u_stride;
        o.W = g.W;
        o.H = g.H;
        o.wF = LF.W;
        o.hF = LF.H;
        o.F = g.F;
        o.pad_left = g.pad_left;
        o.pad_top = g.pad_top;
        o.xmax = upsample_xmax(g);
        o.npw = LF.npw;
        o.nph = LF.nph;
        o.offw = LF.offw;
        o.offh = LF.offh;
        o.steps = LF.steps;
        o.hp = g.ps / 2;
        o.vec_store = ((reinterpret_cast<uintptr_t>(flow) & 15) == 0 && (g.W & 1) == 0) ? 1 : 0;
        o.sc = std::pow(2.0f, (float)g.F);
        o.paper = paper ? 1 : 0;
        o.img0 = img0 + LF.plane_off;
        o.img1 = img1 + LF.plane_off;
        o.plane_stride = g.plane_stride;
        fused_out = dis::output_fits(o) && !vr;  // refined: the finest dense field exists
    }
    if (fused_out) {
        DIS_HIP(dis::launch_output(o, n, s, timing(c, 3)));
    } else {
        if (fast && !c->debug && !vr)  // the level loop skipped the finest densify: do it here
            DIS_HIP(dis::launch_densify(densify_args(c, g.F, img0, img1, pu, dense), n, s));
        const dis::LevelGeom& LF = g.lv[g.F];
        dis::UpsampleArgs u{};
        u.dense = dense + LF.dense_off;
        u.flow = flow;
        u.dense_stride = g.dense_stride;
        u.W = g.W;
        u.H = g.H;
        u.wF = LF.W;
        u.hF = LF.H;
        u.F = g.F;
        u.pad_left = g.pad_left;
        u.pad_top = g.pad_top;
        u.sc = std::pow(2.0f, (float)g.F);
        u.inv_sc = 1.0 / (double)u.sc;
        u.xmax = upsample_xmax(g);
        DIS_HIP(dis::launch_upsample(u, n, s));
    }
    return DIS_OK;
}

// Split n pairs into sub-batches on the context's streams (fork from `s`,
// join back into `s`): pairs are independent, so the latency-bound phases of
// one sub-batch (coarse levels, kernel tails) overlap the others' work. The
// sub-batches run in lockstep (staggered starts, stream priorities and
// uneven splits measured 1-4.5 % slower: DESIGN.md 7), stages issued
// stage-major so every sub-batch's next kernels are queued early.
dis_status run_batches(dis_ctx* c, int n, const uint8_t* I0, const uint8_t* I1, size_t stride,
                       size_t pair_stride, float2* flow, hipStream_t s, bool capturing = false)
{
    // refinement: one stream. Its many short bandwidth-bound kernels stall
    // behind a co-running sub-batch's long search launches (measured on
    // 3840x2160 SLOW, batch 2: 36.3 ms with two streams, 24.1 ms with one).
    const int S = c->p.var_refine_iters > 0 ? 1 : std::min(c->nsub, n);
    c->last_nsub = std::max(S, 1);
    std::vector<int> stages = {kStageFront};
    for (int l = c->g.C; l >= c->g.F; --l) stages.push_back(l);
    stages.push_back(kStageBack);
    if (c->needs_wait(s) && !capturing) DIS_HIP(hipStreamWaitEvent(s, c->done, 0));  // the workspace is free
    if (S <= 1) {
        for (int st : stages) {
            StageRange range(st, 0);
            dis_status r = run_batch(c, 0, n, 0, I0, I1, stride, pair_stride, flow, s, st);
            if (r != DIS_OK) return r;
        }
        c->last_batch = n;
        if (capturing) return DIS_OK;
        DIS_HIP(hipEventRecord(c->done, s));
        c->done_pending = true;
        c->done_stream = s;
        return DIS_OK;
    }
    // Every sub-batch runs on a context-owned stream forked from and joined
    // back into the caller's stream. (Running sub-batch 0 on the caller's stream
    // saves a cross-queue hop, but HIP maps streams onto its few hardware
    // queues in creation order, so whether the caller's stream shares a queue
    // with sub[1] -- serialising the two sub-batches -- depended on how many
    // streams the process had created before: 15k vs 20k pairs/s at 1080p.
    // The context's own streams are created back to back, on distinct queues.)
    // The fork / stages / join sequence as a plan (dis_plan.h): checked against
    // the capture rules before a capture issues any of it -- a plan the HIP
    // runtime cannot capture (an unjoined stream) fails at EndCapture and
    // leaves a stream in capture mode and an invalid graph handle behind
    // (tools/capture_probe.hip) -- then executed op by op.
    const std::vector<dis::PlanOp> plan = dis::batch_plan(S, (int)stages.size());
    if (capturing) {
        const std::string why = dis::check_capture_plan(plan.data(), (int)plan.size(), 1 + S, 1 + S);
        if (!why.empty()) return fail(DIS_ERR_INTERNAL, "batch stream plan cannot be captured: " + why);
    }
    auto stream_of = [&](int x) { return x == 0 ? s : c->sub[x - 1]; };
    auto event_of = [&](int e) { return e == 0 ? c->fork : c->join[e - 1]; };
    const size_t fpp = (size_t)c->g.W * c->g.H;  // float2 per output pair
    for (const dis::PlanOp& o : plan) {
        if (o.kind == dis::kOpRecord) {
            DIS_HIP(hipEventRecord(event_of(o.event), stream_of(o.stream)));
        } else if (o.kind == dis::kOpWait) {
            DIS_HIP(hipStreamWaitEvent(stream_of(o.stream), event_of(o.event), 0));
            if (capturing) {  // the waiting stream must now be in the origin's capture
                hipStreamCaptureStatus cs0, cs1;
                unsigned long long id0 = 0, id1 = 0;
                DIS_HIP(hipStreamGetCaptureInfo(s, &cs0, &id0));
                DIS_HIP(hipStreamGetCaptureInfo(stream_of(o.stream), &cs1, &id1));
                if (cs0 != hipStreamCaptureStatusActive || cs1 != hipStreamCaptureStatusActive || id0 != id1)
                    return fail(DIS_ERR_DEVICE, "graph capture: a sub-batch stream did not join the call's capture");
            }
        } else {
            const int k = o.stream - 1, st = stages[o.stage];
            const int a = (int)((long long)n * k / S), b = (int)((long long)n * (k + 1) / S);
            StageRange range(st, k);
            dis_status r = run_batch(c, k, b - a, a, I0 + (size_t)a * pair_stride, I1 + (size_t)a * pair_stride,
                                     stride, pair_stride, flow + (size_t)a * fpp, stream_of(o.stream), st);
            if (r != DIS_OK) return r;
        }
    }
    c->last_batch = n;
    if (capturing) return DIS_OK;
    DIS_HIP(hipEventRecord(c->done, s));
    c->done_pending = true;
    c->done_stream = s;
    return DIS_OK;
}

// run_batches as a replayed HIP graph (see dis_ctx::MainGraph). Eager when
// graphs are off, under kernel timing (per-dispatch events), debug dumps or
// variational refinement (its own per-level graphs).
dis_status run_batches_graph(dis_ctx* c, int n, const uint8_t* I0, const uint8_t* I1, size_t stride,
                             size_t pair_stride, float2* flow, hipStream_t s)
{
    // eager: graphs off, kernel timing, debug dumps, refinement (its own
    // per-level graphs)
    if (!c->graphs || c->timing || c->debug || c->p.var_refine_iters > 0 || !c->cap) {
        std::lock_guard<std::mutex> lock(pool_mutex(c->device));  // eager enqueue onto the pooled streams
        return run_batches(c, n, I0, I1, stride, pair_stride, flow, s);
    }
    auto key_is = [&](const dis_ctx::MainGraph& G) {
        return G.exec && G.n == n && G.i0 == I0 && G.i1 == I1 && G.flow == flow && G.stride == stride &&
               G.pair_stride == pair_stride && G.nsub == c->nsub && G.precision == c->precision &&
               G.variant == c->variant;
    };
    dis_ctx::MainGraph* G = nullptr;
    for (auto& e : c->mg)
        if (key_is(e)) G = &e;
    if (!G) {
        // victim: an empty slot, else the least recently used exec
        G = &c->mg[0];
        for (auto& e : c->mg) {
            if (!e.exec) {
                G = &e;
                break;
            }
            if (e.used < G->used) G = &e;
        }
        if (G->launched) {  // its last replay may still be in flight: never update under it
            DIS_HIP(hipEventSynchronize(G->last));
            G->launched = false;
        }
        if (!G->last) DIS_HIP(hipEventCreateWithFlags(&G->last, hipEventDisableTiming));
        StageRange range("dis: graph capture");
        hipGraph_t graph = nullptr;
        dis_status r;
        hipError_t e, e0;
        {
            // the capture forks onto the device's pooled sub-batch streams:
            // no other context's eager work may enter them meanwhile
            std::lock_guard<std::mutex> lock(pool_mutex(c->device));
            e0 = hipStreamBeginCapture(c->cap, hipStreamCaptureModeThreadLocal);
            r = e0 == hipSuccess ? run_batches(c, n, I0, I1, stride, pair_stride, flow, c->cap, true) : DIS_OK;
            e = e0 == hipSuccess ? hipStreamEndCapture(c->cap, &graph) : e0;
            // HIP 7.2: a failed EndCapture writes a non-null handle that is not a
            // graph (instantiating it crashed tools/capture_probe, destroying it
            // returns hipErrorIllegalState) -- never touch it
            if (e != hipSuccess) graph = nullptr;
            // and a stream it left unjoined stays in capture mode (mode 5): no
            // later work may go to the pooled streams then
            for (int k = 0; k < dis_ctx::kMaxSub; ++k) {
                hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                if (hipStreamIsCapturing(c->sub[k], &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
                    (void)hipGetLastError();
                    c->graphs = 0;
                    return fail(DIS_ERR_DEVICE, "graph capture left sub-batch stream " + std::to_string(k) +
                                                    " in capture mode (" + hipGetErrorName(e) + ")");
                }
            }
        }
        hipError_t e2 = hipErrorUnknown;
        if (r == DIS_OK && e == hipSuccess) {
            if (G->exec) {  // same topology (same n and sub-batches): update the parameters in place
                hipGraphExecUpdateResult res;
                hipGraphNode_t bad = nullptr;
                e2 = hipGraphExecUpdate(G->exec, graph, &bad, &res);
                if (e2 != hipSuccess) {
                    (void)hipGetLastError();
                    hipGraphExecDestroy(G->exec);
                    G->exec = nullptr;
                }
            }
            if (!G->exec) e2 = hipGraphInstantiate(&G->exec, graph, nullptr, nullptr, 0);
        }
        if (graph) hipGraphDestroy(graph);
        if (r != DIS_OK) {
            // a real error inside the captured enqueue (not an invalidated
            // capture): report it; no eager retry on sub-streams that may still
            // be in a bad capture state
            (void)hipGetLastError();
            if (G->exec) hipGraphExecDestroy(G->exec);
            G->exec = nullptr;
            G->n = -1;
            return r;
        }
        if (e2 != hipSuccess) {
            // The capture was invalidated (e.g. another thread synchronised the
            // device or used the legacy default stream meanwhile) or failed to
            // instantiate: this call runs eagerly -- same results -- and the
            // next call with this key tries to capture again.
            (void)hipGetLastError();
            if (G->exec) hipGraphExecDestroy(G->exec);
            G->exec = nullptr;
            G->n = -1;
            std::lock_guard<std::mutex> lock(pool_mutex(c->device));
            return run_batches(c, n, I0, I1, stride, pair_stride, flow, s);
        }
        G->n = n;
        G->i0 = I0;
        G->i1 = I1;
        G->flow = flow;
        G->stride = stride;
        G->pair_stride = pair_stride;
        G->nsub = c->nsub;
        G->precision = c->precision;
        G->variant = c->variant;
        G->subs = c->last_nsub;
    }
    G->used = ++c->graph_clock;
    c->last_nsub = G->subs;  // a replay runs the sub-batches it was captured with (DIS_STAGE_FALLBACK)
    if (c->needs_wait(s)) DIS_HIP(hipStreamWaitEvent(s, c->done, 0));  // the workspace is free
    {
        StageRange range("dis: graph launch");
        DIS_HIP(hipGraphLaunch(G->exec, s));
    }
    DIS_HIP(hipEventRecord(G->last, s));
    G->launched = true;
    c->last_batch = n;
    DIS_HIP(hipEventRecord(c->done, s));
    c->done_pending = true;
    c->done_stream = s;
    return DIS_OK;
}

// True when [p, p + bytes) lies in one page-locked host allocation
// (hipHostMalloc / hipHostRegister, e.g. torch's pin_memory): the DMA engines
// read or write it directly, no staging copy.
bool host_pinned(const void* p, size_t bytes)
{
    if (!p || !bytes) return false;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error here
        return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
    void *b0 = nullptr, *b1 = nullptr;
    const char* last = static_cast<const char*>(p) + bytes - 1;
    if (hipPointerGetAttribute(&b0, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, const_cast<void*>(p)) != hipSuccess ||
        hipPointerGetAttribute(&b1, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, const_cast<char*>(last)) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return b0 && b0 == b1;
}

// Device slots, streams and the download thread of the host-frame path, made
// on the first host call (device-resident callers never pay for them).
// chunk = 0: about 64 MB of flow per chunk (4 pairs at 1920 x 1080); debug mode
// keeps the whole batch in one chunk (the stage dumps read the last call's
// pairs).
dis_status host_pipe_init(dis_ctx* c, int n)
{
    const size_t frame = (size_t)c->g.W * c->g.H;
    int chunk = c->host_chunk > 0 ? c->host_chunk
                                  : (int)std::max<size_t>(1, (size_t(64) << 20) / (frame * sizeof(float2)));
    if (c->debug) chunk = std::max(chunk, n);
    chunk = std::min(chunk, c->max_batch);
    if (c->hp && c->hp->chunk == chunk) return DIS_OK;
    c->hp.reset();
    auto hp = std::make_unique<HostPipe>();
    hp->chunk = chunk;
    hp->frame = frame;
    hp->device = c->device;
    for (int s = 0; s < 2; ++s) {
        if (hipMalloc(&hp->din[s], 2 * frame * chunk) != hipSuccess ||
            hipMalloc(&hp->dout[s], sizeof(float2) * frame * chunk) != hipSuccess)
            return fail(DIS_ERR_OUT_OF_MEMORY, "host-path device slot allocation failed");
        DIS_HIP(hipEventCreateWithFlags(&hp->up_done[s], hipEventDisableTiming));
        DIS_HIP(hipEventCreateWithFlags(&hp->comp_done[s], hipEventDisableTiming));
        DIS_HIP(hipEventCreateWithFlags(&hp->down_done[s], hipEventDisableTiming));
    }
    DIS_HIP(hipStreamCreateWithFlags(&hp->up, hipStreamNonBlocking));
    DIS_HIP(hipStreamCreateWithFlags(&hp->down, hipStreamNonBlocking));
    HostPipe* raw = hp.get();
    hp->th = std::thread([raw] { raw->run(); });
    c->hp = std::move(hp);
    return DIS_OK;
}

// dis_calc_batch_u8 on host frames and host flow. Chunk j: the calling thread
// uploads it into device slot j % 2 (once the computation of chunk j-2 has
// read that slot), enqueues its computation -- the device path on the
// context's own stream, after the upload and after the download of chunk j-2
// has read the output slot -- and posts its download to the download thread.
// Pageable copies block the thread that issues them until they are done, so
// the upload of chunk j+1 runs while chunk j computes and chunk j-1
// downloads (PCIe is full duplex); page-locked caller buffers (dis_host_alloc,
// hipHostMalloc / hipHostRegister) make every copy asynchronous. The flows are
// the device path's, bit for bit.
dis_status calc_host(dis_ctx* c, int n, const uint8_t* I0, const uint8_t* I1, size_t stride, size_t pair_stride,
                     float* flow)
{
    dis_status st = host_pipe_init(c, n);
    if (st != DIS_OK) return st;
    HostPipe& P = *c->hp;
    const int W = c->g.W, H = c->g.H, chunk = P.chunk;
    const size_t fr = P.frame, fb = fr * sizeof(float2);
    const size_t in_span = (size_t)(n - 1) * pair_stride + (size_t)(H - 1) * stride + W;
    const bool pin_in = host_pinned(I0, in_span) && host_pinned(I1, in_span);
    const bool pin_out = host_pinned(flow, fb * n);
    const hipStream_t s = c->own;
    const int nch = (n + chunk - 1) / chunk;
    const long long base = P.posted;  // jobs of earlier calls (all issued and done)
    auto drain = [&](hipError_t e0) -> dis_status {  // after an error: let the download thread finish
        const hipError_t e1 = P.wait_issued(P.posted);
        const hipError_t e = e0 != hipSuccess ? e0 : e1;
        return fail(DIS_ERR_DEVICE, std::string("host-frame path: ") + hipGetErrorString(e));
    };
    for (int j = 0; j < nch; ++j) {
        const int slot = j & 1, a = j * chunk, m = std::min(chunk, n - a);
        uint8_t* din0 = P.din[slot];
        uint8_t* din1 = P.din[slot] + (size_t)chunk * fr;
        hipError_t e = hipSuccess;
        // upload once the computation of chunk j-2 has read the slot
        if (P.comp_pending[slot]) e = hipStreamWaitEvent(P.up, P.comp_done[slot], 0);
        for (int k = 0; e == hipSuccess && k < m; ++k) {
            e = hipMemcpy2DAsync(din0 + k * fr, W, I0 + (size_t)(a + k) * pair_stride, stride, W, H,
                                 hipMemcpyHostToDevice, P.up);
            if (e == hipSuccess)
                e = hipMemcpy2DAsync(din1 + k * fr, W, I1 + (size_t)(a + k) * pair_stride, stride, W, H,
                                     hipMemcpyHostToDevice, P.up);
        }
        if (e == hipSuccess) e = hipEventRecord(P.up_done[slot], P.up);
        // compute after the upload and after the download of chunk j-2 (its
        // job must have been issued for down_done[slot] to stand for it)
        if (e == hipSuccess) e = hipStreamWaitEvent(s, P.up_done[slot], 0);
        if (e == hipSuccess && P.down_pending[slot]) {
            e = P.wait_issued(base + j - 1);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, P.down_done[slot], 0);
        }
        if (e != hipSuccess) return drain(e);
        // eager enqueue, not a replayed graph: this path is bound by PCIe (a
        // chunk's download takes ~10x its computation), and launching a graph
        // captured here crashed the HIP 7.2 runtime on the host in one call
        // sequence (tools/repro_graph_steps.py EKSFH) that the
        // eager form runs cleanly
        {
            std::lock_guard<std::mutex> lock(pool_mutex(c->device));
            st = run_batches(c, m, din0, din1, (size_t)W, fr, P.dout[slot], s);
        }
        if (st != DIS_OK) {
            drain(hipSuccess);
            return st;
        }
        e = hipEventRecord(P.comp_done[slot], s);
        if (e != hipSuccess) return drain(e);
        P.comp_pending[slot] = true;
        P.down_pending[slot] = true;
        P.post({reinterpret_cast<char*>(flow) + (size_t)a * fb, reinterpret_cast<const char*>(P.dout[slot]), m * fb,
                slot});
    }
    hipError_t e = P.wait_issued(base + nch);
    if (e == hipSuccess) e = hipEventSynchronize(P.down_done[(nch - 1) & 1]);  // page-locked flow: the last copy
    if (e != hipSuccess) return fail(DIS_ERR_DEVICE, std::string("host-frame path: ") + hipGetErrorString(e));
    P.last_chunks = nch;
    P.last_direct_in = pin_in ? 1 : 0;
    P.last_direct_out = pin_out ? 1 : 0;
    return DIS_OK;
}

// Sub-batch streams: one pool per device for the whole process, created
// back to back on first use and never destroyed. HIP maps each new stream
// onto one of its few hardware queues (GPU_MAX_HW_QUEUES = 4) by usage at
// creation time; streams created per context after earlier contexts were
// destroyed landed two sub-batches on one queue (measured: every context
// after the first ran 1080p MEDIUM at 16.5k instead of 20.5k pairs/s with
// 2 streams; 20.2k with 1). Contexts on a device share the pool: work of
// concurrent contexts is ordered within a shared stream, still correct.
bool sub_streams(int device, hipStream_t (&out)[dis_ctx::kMaxSub])
{
    static std::mutex mu;
    static std::map<int, std::vector<hipStream_t>> pools;
    std::lock_guard<std::mutex> lock(mu);
    auto& v = pools[device];
    if (v.empty()) {
        for (int k = 0; k < dis_ctx::kMaxSub; ++k) {
            hipStream_t st = nullptr;
            if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
                for (hipStream_t x : v) hipStreamDestroy(x);
                v.clear();
                return false;
            }
            v.push_back(st);
        }
    }
    for (int k = 0; k < dis_ctx::kMaxSub; ++k) out[k] = v[k];
    return true;
}

// Compat path workspace: one per device for the process, grown on demand.
struct CompatWs {
    std::mutex mu;  // one call at a time on this device's workspace and stream
    float *dx = nullptr, *dy = nullptr, *i1 = nullptr;
    float2 *pu = nullptr, *dense = nullptr;
    int* fb = nullptr;
    size_t planes = 0, u = 0, d = 0, nfb = 0;
    hipStream_t stream = nullptr;
    hipStream_t up = nullptr;                  // plane uploads, level by level
    hipEvent_t level_up[dis::kMaxLevels] = {};  // level l's planes are on the device
    bool reserve(size_t p, size_t nu, size_t nd, size_t nf)
    {
        if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
        if (!up && hipStreamCreateWithFlags(&up, hipStreamNonBlocking) != hipSuccess) return false;
        for (hipEvent_t& e : level_up)
            if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
        if (p > planes) {
            hipFree(dx);
            hipFree(dy);
            hipFree(i1);
            dx = dy = i1 = nullptr;
            planes = 0;
            if (hipMalloc(&dx, sizeof(float) * p) != hipSuccess || hipMalloc(&dy, sizeof(float) * p) != hipSuccess ||
                hipMalloc(&i1, sizeof(float) * p) != hipSuccess)
                return false;
            planes = p;
        }
        if (nu > u) {
            hipFree(pu);
            pu = nullptr;
            u = 0;
            if (hipMalloc(&pu, sizeof(float2) * nu) != hipSuccess) return false;
            u = nu;
        }
        if (nd > d) {
            hipFree(dense);
            dense = nullptr;
            d = 0;
            if (hipMalloc(&dense, sizeof(float2) * nd) != hipSuccess) return false;
            d = nd;
        }
        if (nf > nfb) {
            hipFree(fb);
            fb = nullptr;
            nfb = 0;
            if (hipMalloc(&fb, sizeof(int) * nf) != hipSuccess) return false;
            nfb = nf;
        }
        return true;
    }
};
std::mutex compat_mu;  // guards the map only: calls on different devices run in parallel
CompatWs& compat_ws(int device)
{
    static std::map<int, CompatWs> ws;  // process lifetime (freed by the driver at exit); nodes never move
    std::lock_guard<std::mutex> lock(compat_mu);
    return ws[device];
}

dis::DensifyArgs densify_level(const dis::Geometry& g, int l, float2* pu, float2* dense)
{
    const dis::LevelGeom& L = g.lv[l];
    dis::DensifyArgs d{};
    d.u = pu + L.u_off;
    d.dense = dense + L.dense_off;
    d.u_stride = g.u_stride;
    d.dense_stride = g.dense_stride;
    d.W = L.W;
    d.H = L.H;
    d.ps = g.ps;
    d.steps = L.steps;
    d.npw = L.npw;
    d.nph = L.nph;
    d.offw = L.offw;
    d.offh = L.offh;
    return d;
}

}  // namespace

// ---------------------------------------------------------------------------
// exported C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int dis_abi_version(void) { return DIS_ABI_VERSION; }
const char* dis_build_kind(void) { return "product"; }

const char* dis_last_error(void) { return g_err.c_str(); }

dis_status dis_preset_params(dis_preset preset, int width, int height, dis_params* out)
{
    if (!out) return fail(DIS_ERR_INVALID_ARGUMENT, "out is null");
    if (width < 1 || height < 1) return fail(DIS_ERR_INVALID_ARGUMENT, "width and height must be >= 1");
    dis_params p{};
    p.patch_size = 8;
    p.patch_normalization = 1;
    p.var_refine_iters = 0;
    switch (preset) {
        case DIS_PRESET_ULTRAFAST: p.patch_overlap = 0.5f; p.iterations = 12; p.finest_scale = 2; break;
        case DIS_PRESET_FAST: p.patch_overlap = 0.5f; p.iterations = 16; p.finest_scale = 2; break;
        case DIS_PRESET_MEDIUM: p.patch_overlap = 0.625f; p.iterations = 25; p.finest_scale = 1; break;
        case DIS_PRESET_SLOW:  // + variational refinement (BASELINE config 5; not in the reference)
            p.patch_overlap = 0.75f; p.iterations = 128; p.finest_scale = 0; p.var_refine_iters = 3; break;
        case DIS_PRESET_REFERENCE:
            // CLI defaults, src/main.cpp:66-71
            p.patch_overlap = 0.7f; p.iterations = 1000; p.finest_scale = 0; p.coarsest_scale = 3;
            *out = p;
            return DIS_OK;
        default: return fail(DIS_ERR_INVALID_ARGUMENT, "unknown preset");
    }
    // C = auto: integer division in min(W,H)/ps
    const int mx = std::max(width, height), mn = std::min(width, height);
    int c1 = (int)(std::log2((double)mx / (4.0 * p.patch_size)) + 0.5);
    int c2 = (mn / p.patch_size) > 0 ? (int)std::log2((double)(mn / p.patch_size)) : 0;
    int C = std::max(0, std::min(c1, c2));
    p.coarsest_scale = C;
    p.finest_scale = std::min(p.finest_scale, C);
    *out = p;
    return DIS_OK;
}

dis_status dis_validate_params(const dis_params* params, int width, int height)
{
    return check_params(params, width, height);
}

dis_status dis_workload_info(const dis_params* params, int width, int height, dis_workload* out)
{
    dis_status st = check_params(params, width, height);
    if (st != DIS_OK) return st;
    if (!out) return fail(DIS_ERR_INVALID_ARGUMENT, "out is null");
    dis::Geometry g;
    if (!dis::make_geometry(*params, width, height, &g)) return fail(DIS_ERR_INVALID_ARGUMENT, "bad geometry");
    // SURVEY.md 8d fixed formula
    double B = 2.0 * width * height;
    long long patches = 0, updates = 0;
    for (int l = 0; l <= g.C; ++l) B += 8.0 * g.lv[l].W * g.lv[l].H;
    for (int l = g.F; l <= g.C; ++l) {
        const double px = (double)g.lv[l].W * g.lv[l].H;
        B += 8.0 * px;                               // frame-0 dx, dy
        B += 16.0 * px + 16.0 * g.lv[l].n + 8.0 * px;  // search reads + u + dense write
        patches += g.lv[l].n;
        updates += (long long)g.lv[l].n * (g.iters + 1);
    }
    for (int l = g.F; l < g.C; ++l) B += 8.0 * g.lv[l + 1].W * g.lv[l + 1].H;
    if (g.F > 0) B += 8.0 * g.lv[g.F].W * g.lv[g.F].H + 8.0 * width * height;
    out->padded_width = g.Wp;
    out->padded_height = g.Hp;
    out->steps = g.steps;
    out->patches = patches;
    out->updates = updates;
    out->algorithmic_bytes = B;
    const dis::LevelGeom& LF = g.lv[g.F];
    out->search_bytes_finest = 16.0 * LF.W * LF.H + 16.0 * LF.n;
    double sb = 0.0;
    for (int l = g.F; l <= g.C; ++l) {
        sb += 16.0 * g.lv[l].W * g.lv[l].H + 16.0 * g.lv[l].n;
        if (l < g.C) sb += 8.0 * g.lv[l + 1].W * g.lv[l + 1].H;
    }
    out->search_bytes_all = sb;
    out->search_launches = g.C - g.F + 1;
    // algorithmic f32 operations per patch (each add/sub/mul/div = 1): Sobel
    // gradients ~10/pixel, Hessian 3 dot products, 2x2 LU; per update: bilinear
    // warp 7/pixel (4 mul + 3 add), mean normalisation 2/pixel, 2 dot products,
    // solve + update + outlier test ~12 (src/patch.cpp:31-267)
    const double N = (double)g.ps * g.ps;
    const double per_update = 7.0 * N + (g.norm ? 2.0 * N : 0.0) + 2.0 * (2.0 * N - 1.0) + 14.0;
    const double per_patch = 10.0 * N + 3.0 * (2.0 * N - 1.0) + 6.0 + (g.iters + 1) * per_update;
    out->patches_finest = LF.n;
    out->search_flops_finest = (double)LF.n * per_patch;
    return DIS_OK;
}

dis_status dis_create(dis_ctx** out, const dis_params* params, int width, int height, int max_batch,
                      int device)
{
    if (!out) return fail(DIS_ERR_INVALID_ARGUMENT, "out is null");
    *out = nullptr;
    dis_status st = check_params(params, width, height);
    if (st != DIS_OK) return st;
    if (max_batch < 1) return fail(DIS_ERR_INVALID_ARGUMENT, "max_batch must be >= 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(DIS_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(DIS_ERR_INVALID_ARGUMENT, "device index out of range");
    dis_ctx* c = new (std::nothrow) dis_ctx();
    if (!c) return fail(DIS_ERR_OUT_OF_MEMORY, "host allocation failed");
    c->p = *params;
    c->device = device;
    c->max_batch = max_batch;
    if (!dis::make_geometry(*params, width, height, &c->g)) {
        delete c;
        return fail(DIS_ERR_INVALID_ARGUMENT, "bad geometry");
    }
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return fail(DIS_ERR_DEVICE, "hipSetDevice failed");
    }
    const dis::Geometry& g = c->g;
    const size_t B = (size_t)max_batch;
    const size_t plane = sizeof(float) * (size_t)g.plane_stride * B;
    bool ok = hipMalloc(&c->img0, plane) == hipSuccess && hipMalloc(&c->img1, plane) == hipSuccess &&
              hipMalloc(&c->dx, plane) == hipSuccess && hipMalloc(&c->dy, plane) == hipSuccess &&
              hipMalloc(&c->pu, sizeof(float2) * (size_t)g.u_stride * B) == hipSuccess &&
              hipMalloc(&c->dense, sizeof(float2) * (size_t)g.dense_stride * B) == hipSuccess &&
              hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->done, hipEventDisableTiming) == hipSuccess;
    if (ok) {
        size_t off = (size_t)dis_ctx::kMaxSub * kFbCounters;
        for (int k = 0; k < dis_ctx::kMaxSub; ++k)
            for (int l = 0; l <= g.C; ++l) {
                c->fb_list_off[k][l] = off;
                off += (size_t)((g.lv[l].npw + 7) / 8) * ((g.lv[l].nph + 7) / 8) * B;  // 8x8 blocks (the most)
            }
        ok = hipMalloc(&c->fb, sizeof(int) * off) == hipSuccess &&
             hipMemset(c->fb, 0, sizeof(int) * dis_ctx::kMaxSub * kFbCounters) == hipSuccess;
    }
    if (ok && params->var_refine_iters > 0) {
        c->vr_plane = (long long)g.lv[g.F].W * g.lv[g.F].H;  // the largest refined level
        ok = hipMalloc(&c->vr_ws, sizeof(float) * dis::kVarRefPlanes * c->vr_plane * B) == hipSuccess;
    }
    ok = ok && sub_streams(device, c->sub);
    for (int k = 0; ok && k < dis_ctx::kMaxSub; ++k)
        ok = hipEventCreateWithFlags(&c->join[k], hipEventDisableTiming) == hipSuccess;
    // The capture-only stream exists only under refinement and is created last:
    // HIP assigns streams to its (GPU_MAX_HW_QUEUES = 4) hardware queues round
    // robin at creation, and an extra stream created before sub[] shifted
    // sub[1] onto the caller's (null stream's) queue, serialising the two
    // sub-batches (measured: 20.1k -> 15.5k pairs/s at 1080p MEDIUM).
    if (ok) ok = hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        free_ws(c);
        for (int k = 0; k < dis_ctx::kMaxSub; ++k)
            if (c->join[k]) hipEventDestroy(c->join[k]);
        if (c->fork) hipEventDestroy(c->fork);
        if (c->done) hipEventDestroy(c->done);
        if (c->cap) hipStreamDestroy(c->cap);
        if (c->own) hipStreamDestroy(c->own);
        delete c;
        return fail(DIS_ERR_OUT_OF_MEMORY, "device workspace allocation failed");
    }
    *out = c;
    return DIS_OK;
}

dis_status dis_destroy(dis_ctx* c)
{
    if (!c) return DIS_OK;
    hipSetDevice(c->device);
    if (c->own) hipStreamSynchronize(c->own);
    if (c->done_pending) hipEventSynchronize(c->done);  // the last call, on whatever stream it ran
    for (int k = 0; k < dis_ctx::kMaxSub; ++k)  // the streams are shared (process pool): wait for this
        if (c->join[k]) hipEventSynchronize(c->join[k]);  // context's last join, not the stream
    free_ws(c);
    for (hipEvent_t e : c->pool) hipEventDestroy(e);
    for (int k = 0; k < dis_ctx::kMaxSub; ++k)
        if (c->join[k]) hipEventDestroy(c->join[k]);
    if (c->fork) hipEventDestroy(c->fork);
    if (c->done) hipEventDestroy(c->done);
    for (auto& row : c->vrg)
        for (auto& G : row)
            if (G.exec) hipGraphExecDestroy(G.exec);
    for (auto& G : c->mg) {
        if (G.exec) hipGraphExecDestroy(G.exec);
        if (G.last) hipEventDestroy(G.last);
    }
    if (c->cap) hipStreamDestroy(c->cap);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
    return DIS_OK;
}

dis_status dis_calc_batch_u8(dis_ctx* c, int n, const uint8_t* I0, const uint8_t* I1, size_t stride,
                             size_t pair_stride, float* flow, dis_mem where, void* stream)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    if (!I0 || !I1 || !flow) return fail(DIS_ERR_INVALID_ARGUMENT, "null frame or flow pointer");
    if (n < 1 || n > c->max_batch) return fail(DIS_ERR_INVALID_ARGUMENT, "n must be in [1, max_batch]");
    const int W = c->g.W, H = c->g.H;
    if (stride == 0) stride = (size_t)W;
    if (stride < (size_t)W) return fail(DIS_ERR_INVALID_ARGUMENT, "stride < width");
    if (pair_stride == 0) pair_stride = stride * H;
    if (n > 1 && pair_stride < stride * H) return fail(DIS_ERR_INVALID_ARGUMENT, "pair_stride too small");
    DIS_HIP(hipSetDevice(c->device));
    if (where == DIS_MEM_DEVICE) {
        return run_batches_graph(c, n, I0, I1, stride, pair_stride, reinterpret_cast<float2*>(flow),
                                 reinterpret_cast<hipStream_t>(stream));
    }
    if (where != DIS_MEM_HOST) return fail(DIS_ERR_INVALID_ARGUMENT, "bad dis_mem");
    return calc_host(c, n, I0, I1, stride, pair_stride, flow);
}

dis_status dis_set_host_pipeline(dis_ctx* c, int chunk_pairs)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    if (chunk_pairs < 0) return fail(DIS_ERR_INVALID_ARGUMENT, "chunk_pairs must be >= 0 (0 = auto)");
    DIS_HIP(hipSetDevice(c->device));
    c->hp.reset();  // rebuilt on the next host call (host calls are synchronous: nothing in flight)
    c->host_chunk = chunk_pairs;
    return DIS_OK;
}

dis_status dis_host_pipeline_info(dis_ctx* c, dis_host_info* out)
{
    if (!c || !out) return fail(DIS_ERR_INVALID_ARGUMENT, "null argument");
    std::memset(out, 0, sizeof(*out));
    if (c->hp) {
        out->chunk_pairs = c->hp->chunk;
        out->last_chunks = c->hp->last_chunks;
        out->last_direct_in = c->hp->last_direct_in;
        out->last_direct_out = c->hp->last_direct_out;
    }
    return DIS_OK;
}

dis_status dis_host_alloc(size_t bytes, void** out)
{
    if (!out) return fail(DIS_ERR_INVALID_ARGUMENT, "out is null");
    *out = nullptr;
    if (!bytes) return fail(DIS_ERR_INVALID_ARGUMENT, "bytes must be > 0");
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return fail(DIS_ERR_OUT_OF_MEMORY, "page-locked host allocation failed");
    }
    return DIS_OK;
}

dis_status dis_host_free(void* p)
{
    if (p && hipHostFree(p) != hipSuccess) return fail(DIS_ERR_INVALID_ARGUMENT, "not a dis_host_alloc pointer");
    return DIS_OK;
}

dis_status dis_calc_u8(dis_ctx* c, const uint8_t* I0, const uint8_t* I1, size_t stride, float* flow,
                       dis_mem where, void* stream)
{
    return dis_calc_batch_u8(c, 1, I0, I1, stride, 0, flow, where, stream);
}

dis_status dis_set_debug(dis_ctx* c, int enable)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    c->debug = enable ? 1 : 0;  // this build always materialises every stage
    return DIS_OK;
}

dis_status dis_set_concurrency(dis_ctx* c, int streams)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    if (streams < 1 || streams > dis_ctx::kMaxSub)
        return fail(DIS_ERR_INVALID_ARGUMENT, "streams must be in [1, 8]");
    c->nsub = streams;
    return DIS_OK;
}

dis_status dis_set_graphs(dis_ctx* c, int enable)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    c->graphs = enable ? 1 : 0;
    return DIS_OK;
}

dis_status dis_set_precision(dis_ctx* c, int mode)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    if (mode != DIS_PRECISION_EXACT && mode != DIS_PRECISION_FMA)
        return fail(DIS_ERR_INVALID_ARGUMENT, "precision must be DIS_PRECISION_EXACT or DIS_PRECISION_FMA");
    c->precision = mode;
    return DIS_OK;
}

dis_status dis_set_kernel_variant(dis_ctx* c, int variant)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    if (variant < 0 || variant > 9 || variant == 7 || variant == 8)
        return fail(DIS_ERR_INVALID_ARGUMENT, "variant must be 0..6 or 9 (7 and 8 were removed in ABI v7)");
    c->variant = variant;
    return DIS_OK;
}

dis_status dis_stage_size(dis_ctx* c, int stage, int level, size_t* count)
{
    if (!c || !count) return fail(DIS_ERR_INVALID_ARGUMENT, "null argument");
    const dis::Geometry& g = c->g;
    if (level < 0 || level > g.C) return fail(DIS_ERR_INVALID_ARGUMENT, "level out of range");
    const dis::LevelGeom& L = g.lv[level];
    switch (stage) {
        case DIS_STAGE_IMG0:
        case DIS_STAGE_IMG1:
        case DIS_STAGE_DX0:
        case DIS_STAGE_DY0: *count = (size_t)L.W * L.H; return DIS_OK;
        case DIS_STAGE_PATCH_U: *count = (size_t)L.n * 2; return DIS_OK;
        case DIS_STAGE_DENSE: *count = (size_t)L.W * L.H * 2; return DIS_OK;
        case DIS_STAGE_FALLBACK: *count = 1; return DIS_OK;
        default: return fail(DIS_ERR_INVALID_ARGUMENT, "unknown stage");
    }
}

dis_status dis_debug_dump(dis_ctx* c, int stage, int level, int pair, float* dst, size_t count)
{
    size_t need = 0;
    dis_status st = dis_stage_size(c, stage, level, &need);
    if (st != DIS_OK) return st;
    if (!dst || count < need) return fail(DIS_ERR_INVALID_ARGUMENT, "dst null or too small");
    if (pair < 0 || pair >= c->last_batch) return fail(DIS_ERR_INVALID_ARGUMENT, "pair not in last batch");
    const dis::Geometry& g = c->g;
    const dis::LevelGeom& L = g.lv[level];
    if ((stage == DIS_STAGE_DX0 || stage == DIS_STAGE_DY0 || stage == DIS_STAGE_PATCH_U ||
         stage == DIS_STAGE_DENSE) && level < g.F)
        return fail(DIS_ERR_INVALID_ARGUMENT, "stage not computed below finest_scale");
    DIS_HIP(hipSetDevice(c->device));
    DIS_HIP(hipDeviceSynchronize());
    if (stage == DIS_STAGE_FALLBACK) {  // blocks the level's tile search listed for k_search8_fb, all sub-batches
        std::vector<int> cnt((size_t)c->last_nsub);
        for (int k = 0; k < c->last_nsub; ++k)
            DIS_HIP(hipMemcpy(&cnt[k], c->fb + (size_t)k * kFbCounters + level, sizeof(int), hipMemcpyDeviceToHost));
        long long t = 0;
        for (int v : cnt) t += v;
        *dst = (float)t;
        return DIS_OK;
    }
    const void* src = nullptr;
    switch (stage) {
        case DIS_STAGE_IMG0: src = c->img0 + pair * g.plane_stride + L.plane_off; break;
        case DIS_STAGE_IMG1: src = c->img1 + pair * g.plane_stride + L.plane_off; break;
        case DIS_STAGE_DX0: src = c->dx + pair * g.plane_stride + L.plane_off; break;
        case DIS_STAGE_DY0: src = c->dy + pair * g.plane_stride + L.plane_off; break;
        case DIS_STAGE_PATCH_U: src = c->pu + pair * g.u_stride + L.u_off; break;
        case DIS_STAGE_DENSE: src = c->dense + pair * g.dense_stride + L.dense_off; break;
    }
    DIS_HIP(hipMemcpy(dst, src, sizeof(float) * need, hipMemcpyDeviceToHost));
    return DIS_OK;
}

dis_status dis_set_kernel_timing(dis_ctx* c, int enable)
{
    if (!c) return fail(DIS_ERR_INVALID_ARGUMENT, "ctx is null");
    DIS_HIP(hipSetDevice(c->device));
    if (enable && c->pool.empty()) {
        c->pool.resize(8192);
        for (auto& e : c->pool) DIS_HIP(hipEventCreate(&e));
    }
    if (enable && !c->timing) {  // (re)enabling starts a fresh measurement
        for (auto& r : c->recs) DIS_HIP(hipEventSynchronize(r.b));
        c->recs.clear();
        c->pool_next = 0;
        for (int k = 0; k < dis_ctx::kKinds; ++k) {
            c->launches[k] = 0;
            c->total_ms[k] = 0.0;
        }
        c->dropped = 0;
    }
    c->timing = enable ? 1 : 0;
    return DIS_OK;
}

dis_status dis_kernel_time(dis_ctx* c, int kernel, int* launches, double* total_ms)
{
    if (!c || kernel < 0 || kernel >= dis_ctx::kKinds) return fail(DIS_ERR_INVALID_ARGUMENT, "bad argument");
    DIS_HIP(hipSetDevice(c->device));
    for (auto& r : c->recs) {
        DIS_HIP(hipEventSynchronize(r.b));
        float ms = 0.f;
        DIS_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        if (r.kind >= 0 && r.kind < dis_ctx::kKinds) {
            c->launches[r.kind] += 1;
            c->total_ms[r.kind] += ms;
        }
    }
    c->recs.clear();
    c->pool_next = 0;
    if (c->dropped) return fail(DIS_ERR_DEVICE, "kernel timing records were dropped (event creation failed)");
    if (launches) *launches = c->launches[kernel];
    if (total_ms) *total_ms = c->total_ms[kernel];
    return DIS_OK;
}

// Compat path: OpticalFlowClass(...) semantics over caller-padded host pyramids.
dis_status dis_flow_from_pyramids(const float* const* img_first, const float* const* img_first_dx,
                                  const float* const* img_first_dy, const float* const* img_second,
                                  const float* const* img_second_dx, const float* const* img_second_dy,
                                  int img_padding, float* outflow, int width, int height, int coarsest,
                                  int finest, int iterations, int patch_size, float patch_overlap,
                                  int patch_normalization, int device)
{
    (void)img_first;      // the template T is never used by the reference (Q2)
    (void)img_second_dx;  // frame-2 gradients are never read (Q15)
    (void)img_second_dy;
    if (!img_first_dx || !img_first_dy || !img_second || !outflow)
        return fail(DIS_ERR_INVALID_ARGUMENT, "null pyramid or output pointer");
    dis_params p{};
    p.coarsest_scale = coarsest;
    p.finest_scale = finest;
    p.patch_size = patch_size;
    p.iterations = iterations;
    p.patch_overlap = patch_overlap;
    p.patch_normalization = patch_normalization ? 1 : 0;
    dis_status st = check_params(&p, width, height);
    if (st != DIS_OK) return st;
    if ((width % (1 << coarsest)) || (height % (1 << coarsest)))
        return fail(DIS_ERR_INVALID_ARGUMENT, "width/height must be multiples of 2^coarsest");
    if (img_padding < patch_size)
        return fail(DIS_ERR_INVALID_ARGUMENT, "img_padding must be >= patch_size");
    for (int l = finest; l <= coarsest; ++l)
        if (!img_first_dx[l] || !img_first_dy[l] || !img_second[l])
            return fail(DIS_ERR_INVALID_ARGUMENT, "null plane in pyramid");
    dis::Geometry g;
    if (!dis::make_geometry(p, width, height, &g)) return fail(DIS_ERR_INVALID_ARGUMENT, "bad geometry");
    // physically padded plane stacks
    long long poff[dis::kMaxLevels], tot = 0;
    for (int l = 0; l <= g.C; ++l) {
        poff[l] = tot;
        tot += (long long)(g.lv[l].W + 2 * img_padding) * (g.lv[l].H + 2 * img_padding);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(DIS_ERR_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(DIS_ERR_INVALID_ARGUMENT, "device index out of range");
    DIS_HIP(hipSetDevice(device));
    // per-device workspace, grown on demand and kept for the next call (the
    // reference constructs one OpticalFlowClass per frame pair: a malloc/free
    // per call would dominate)
    size_t fb_n = dis::kMaxLevels;
    for (int l = g.F; l <= g.C; ++l) fb_n += (size_t)((g.lv[l].npw + 7) / 8) * ((g.lv[l].nph + 7) / 8);
    CompatWs& w = compat_ws(device);
    std::lock_guard<std::mutex> lock(w.mu);
    if (!w.reserve(tot, g.u_stride, g.dense_stride, fb_n)) return fail(DIS_ERR_OUT_OF_MEMORY, "device allocation failed");
    hipStream_t s = w.stream;
    const bool fast = g.ps == 8;
    // The planes go up level by level, coarsest first, on a stream of their
    // own; level l's search waits only for level l's planes. A pageable upload
    // returns when it is done, so the finer (larger) levels' uploads run while
    // the coarser levels search.
    auto upload = [&](int l) {
        const size_t bytes = sizeof(float) * (size_t)(g.lv[l].W + 2 * img_padding) * (g.lv[l].H + 2 * img_padding);
        if (hipMemcpyAsync(w.dx + poff[l], img_first_dx[l], bytes, hipMemcpyHostToDevice, w.up) != hipSuccess ||
            hipMemcpyAsync(w.dy + poff[l], img_first_dy[l], bytes, hipMemcpyHostToDevice, w.up) != hipSuccess ||
            hipMemcpyAsync(w.i1 + poff[l], img_second[l], bytes, hipMemcpyHostToDevice, w.up) != hipSuccess ||
            hipEventRecord(w.level_up[l], w.up) != hipSuccess || hipStreamWaitEvent(s, w.level_up[l], 0) != hipSuccess)
            return fail(DIS_ERR_DEVICE, "pyramid upload failed");
        return DIS_OK;
    };
    // (the previous call's searches have read the workspace: `up` follows `s`)
    DIS_HIP(hipEventRecord(w.level_up[g.C], s));
    DIS_HIP(hipStreamWaitEvent(w.up, w.level_up[g.C], 0));
    if (fast) DIS_HIP(hipMemsetAsync(w.fb, 0, sizeof(int) * dis::kMaxLevels, s));
    size_t fb_off = dis::kMaxLevels;
    for (int l = g.C; l >= g.F; --l) {
        const dis::LevelGeom& L = g.lv[l];
        if (dis_status us = upload(l); us != DIS_OK) return us;
        if (fast) {  // the patch_size-8 search on the caller's planes (Search8Args.gdx_plane)
            dis::Search8Args b{};
            b.img1 = w.i1;
            b.gdx_plane = w.dx;
            b.gdy_plane = w.dy;
            b.pad = img_padding;
            b.u_coarse = (l < g.C) ? w.pu + g.lv[l + 1].u_off : nullptr;
            b.u_out = w.pu + L.u_off;
            b.plane_stride = tot;
            b.plane_off = poff[l];
            b.u_stride = g.u_stride;
            b.W = L.W;
            b.H = L.H;
            b.steps = L.steps;
            b.npw = L.npw;
            b.nph = L.nph;
            b.offw = L.offw;
            b.offh = L.offh;
            if (l < g.C) {
                b.c_npw = g.lv[l + 1].npw;
                b.c_nph = g.lv[l + 1].nph;
                b.c_offw = g.lv[l + 1].offw;
                b.c_offh = g.lv[l + 1].offh;
            }
            b.tmp_lb = L.tmp_lb;
            b.tmp_ub_w = L.tmp_ub_w;
            b.tmp_ub_h = L.tmp_ub_h;
            b.thr_sq = sqrt_threshold((float)g.ps / 2);
            b.lanes_per_patch = search8_lanes(0, (long long)L.npw * L.nph, L.steps) == 8 ? 8 : 2;
            b.tile_stride = dis::search8_tile_stride(L.steps, b.lanes_per_patch);
            b.quad = dis::search8_tile_quad(L.steps, b.lanes_per_patch);
            b.fb_count = w.fb + l;
            b.fb_list = w.fb + fb_off;
            fb_off += (size_t)((L.npw + 7) / 8) * ((L.nph + 7) / 8);
            b.iters = g.iters;
            b.norm = g.norm;
            if (dis::launch_search8(b, 1, s) != hipSuccess) return fail(DIS_ERR_DEVICE, "search launch failed");
            continue;
        }
        dis::SearchArgs a{};
        a.img1 = w.i1;
        a.dx = w.dx;
        a.dy = w.dy;
        a.dense_coarse = (l < g.C) ? w.dense + g.lv[l + 1].dense_off : nullptr;
        a.u_out = w.pu + L.u_off;
        a.plane_stride = tot;
        a.plane_off = poff[l];
        a.dense_stride = g.dense_stride;
        a.u_stride = g.u_stride;
        a.phys_pad = img_padding;
        a.W = L.W;
        a.H = L.H;
        a.steps = L.steps;
        a.npw = L.npw;
        a.nph = L.nph;
        a.offw = L.offw;
        a.offh = L.offh;
        a.n = L.n;
        a.tmp_lb = L.tmp_lb;
        a.tmp_ub_w = L.tmp_ub_w;
        a.tmp_ub_h = L.tmp_ub_h;
        a.outlier = (float)g.ps / 2;
        a.iters = g.iters;
        a.norm = g.norm;
        if (dis::launch_search_generic(a, g.ps, 1, s) != hipSuccess) return fail(DIS_ERR_DEVICE, "search launch failed");
        if (l > g.F && dis::launch_densify(densify_level(g, l, w.pu, w.dense), 1, s) != hipSuccess)
            return fail(DIS_ERR_DEVICE, "densify launch failed");
    }
    // the finest level's dense flow (src/patch_grid.cpp:121-182) is the output
    if (dis::launch_densify(densify_level(g, g.F, w.pu, w.dense), 1, s) != hipSuccess)
        return fail(DIS_ERR_DEVICE, "densify launch failed");
    const dis::LevelGeom& LF = g.lv[g.F];
    if (hipMemcpyAsync(outflow, w.dense + LF.dense_off, sizeof(float2) * LF.W * LF.H, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail(DIS_ERR_DEVICE, "result download failed");
    return DIS_OK;
}

dis_status dis_flow_color(const float* flow, int n, int width, int height, float maxmotion, uint8_t* bgr,
                          dis_mem where, void* stream, int device)
{
    if (!flow || !bgr) return fail(DIS_ERR_INVALID_ARGUMENT, "null pointer");
    if (n < 1 || width < 1 || height < 1) return fail(DIS_ERR_INVALID_ARGUMENT, "n, width, height must be >= 1");
    if (where != DIS_MEM_HOST && where != DIS_MEM_DEVICE) return fail(DIS_ERR_INVALID_ARGUMENT, "bad dis_mem");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(DIS_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(DIS_ERR_INVALID_ARGUMENT, "device index out of range");
    DIS_HIP(hipSetDevice(device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t fbytes = sizeof(float) * 2 * (size_t)width * height * n;
    const size_t cbytes = (size_t)3 * width * height * n;
    if (where == DIS_MEM_DEVICE) {
        unsigned int* maxbits = nullptr;
        DIS_HIP(hipMallocAsync(reinterpret_cast<void**>(&maxbits), sizeof(unsigned int) * dis::flow_color_ws_words(n), s));
        const hipError_t e = dis::launch_flow_color(flow, n, width, height, maxmotion, bgr, maxbits, s);
        DIS_HIP(hipFreeAsync(maxbits, s));
        DIS_HIP(e);
        return DIS_OK;
    }
    float* dflow = nullptr;
    uint8_t* dbgr = nullptr;
    unsigned int* maxbits = nullptr;
    dis_status rc = DIS_OK;
    if (hipMalloc(&dflow, fbytes) != hipSuccess || hipMalloc(&dbgr, cbytes) != hipSuccess ||
        hipMalloc(&maxbits, sizeof(unsigned int) * dis::flow_color_ws_words(n)) != hipSuccess) {
        rc = fail(DIS_ERR_OUT_OF_MEMORY, "device allocation failed");
    } else if (hipMemcpyAsync(dflow, flow, fbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
               dis::launch_flow_color(dflow, n, width, height, maxmotion, dbgr, maxbits, s) != hipSuccess ||
               hipMemcpyAsync(bgr, dbgr, cbytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipStreamSynchronize(s) != hipSuccess) {
        rc = fail(DIS_ERR_DEVICE, "flow colour coding failed");
    }
    hipFree(dflow);
    hipFree(dbgr);
    hipFree(maxbits);
    return rc;
}

}  // extern "C"
