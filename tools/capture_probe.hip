// capture_probe.hip -- which cross-stream event patterns inside a HIP stream
// capture (hipStreamBeginCapture(ThreadLocal)) the runtime handles, and which
// it rejects or crashes on. Reduces the r05 host SIGSEGV (the
// finest level as one launch over both sub-batches, sub-batch 0 waiting on the
// sibling sub-batch streams' events during a graph capture) to single API
// sequences. One mode per process (a crash ends only that mode):
//
//   capture_probe <mode>
//   1  fork cap -> s0, s1; kernels; join both into cap            (the product's plan)
//   2  + sibling wait: s0 waits on an event recorded on s1 in the capture,
//      then s1 waits on an event recorded on s0 (the r05 merged pattern)
//   3  s0 waits on an event last recorded on s1 BEFORE the capture began
//      (s1 never joined this capture): a stale, uncaptured event
//   4  s0 waits on an event recorded on s1 in the capture, s1 joined, but the
//      same event object is re-recorded on s1 afterwards (event reuse)
//   5  capture ends with s1 forked but never joined back (unjoined)
//   6  an uncaptured stream waits on an event recorded inside the capture
//   7  s1 joined back only through s0 (s0 waits on s1's last record, the
//      origin waits on s0's): a transitive join
//   8  as 5, then hipGraphDestroy of the handle the failed EndCapture wrote
//      (what run_batches_graph did with it until r06)
//   9  as 5, then a kernel launch and a synchronise on the unjoined stream
//  10  a barrier between the siblings, then the join with the SAME events:
//      s0 records j0, s1 records j1, each waits on the other's, more kernels,
//      then j0 / j1 are recorded again and the origin waits on them (the
//      product's plan with a mid-call sub-batch barrier)
//  11  as 10 with distinct events for the barrier and the join
//  12  as 10 with the product's shape: 5 kernels per stream before the
//      barrier and 7 after, each with a 256-byte argument block
//  13  as 12 with distinct barrier events
//
// Prints each call's status; exit 0 when the sequence ran to the end (whatever
// the statuses), so a host crash shows as the process's signal.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_add(float* p, float v)
{
    p[threadIdx.x] += v;
}

struct BigArgs {
    float* p;
    float v;
    int pad[60];
};
__global__ void k_big(BigArgs a)
{
    a.p[threadIdx.x] += a.v + (float)a.pad[threadIdx.x & 31];
}

#define CALL(x)                                                                       \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        std::printf("  %-60s -> %s\n", #x, hipGetErrorName(e_));                      \
        std::fflush(stdout);                                                          \
    } while (0)

static void status(const char* what, hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipError_t e = hipStreamGetCaptureInfo(s, &st, &id);
    std::printf("  capture status of %-6s: %d (id %llu, %s)\n", what, (int)st, id, hipGetErrorName(e));
    std::fflush(stdout);
}

int main(int argc, char** argv)
{
    const int mode = argc > 1 ? std::atoi(argv[1]) : 1;
    std::printf("mode %d\n", mode);
    float* d = nullptr;
    hipMalloc(&d, 256 * sizeof(float));
    hipMemset(d, 0, 256 * sizeof(float));
    hipStream_t cap, s0, s1, other;
    hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&other, hipStreamNonBlocking);
    hipEvent_t fork, j0, j1, mid0, mid1;
    for (hipEvent_t* e : {&fork, &j0, &j1, &mid0, &mid1}) hipEventCreateWithFlags(e, hipEventDisableTiming);
    if (mode == 3) {  // an eager record on s1 before the capture
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s1, d, 1.f);
        CALL(hipEventRecord(mid1, s1));
        CALL(hipStreamSynchronize(s1));
    }
    CALL(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    CALL(hipEventRecord(fork, cap));
    CALL(hipStreamWaitEvent(s0, fork, 0));
    if (mode != 3) CALL(hipStreamWaitEvent(s1, fork, 0));
    status("cap", cap);
    status("s0", s0);
    status("s1", s1);
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s0, d, 1.f);
    if (mode != 3) hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s1, d + 64, 1.f);
    if (mode == 2 || mode == 4) {
        CALL(hipEventRecord(mid1, s1));
        CALL(hipStreamWaitEvent(s0, mid1, 0));  // sibling-to-sibling
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s0, d + 128, 2.f);
        if (mode == 2) {
            CALL(hipEventRecord(mid0, s0));
            CALL(hipStreamWaitEvent(s1, mid0, 0));
            hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s1, d + 192, 2.f);
        }
    }
    if (mode == 3) {
        CALL(hipStreamWaitEvent(s0, mid1, 0));  // stale event, s1 outside the capture
        status("s1", s1);
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s0, d + 128, 2.f);
    }
    BigArgs ba{};
    ba.v = 0.f;
    if (mode == 12 || mode == 13) {
        for (int k = 0; k < 5; ++k) {
            ba.p = d;
            hipLaunchKernelGGL(k_big, dim3(4), dim3(64), 0, s0, ba);
            ba.p = d + 64;
            hipLaunchKernelGGL(k_big, dim3(4), dim3(64), 0, s1, ba);
        }
    }
    if (mode >= 10 && mode <= 13) {
        hipEvent_t b0 = (mode == 10 || mode == 12) ? j0 : mid0, b1 = (mode == 10 || mode == 12) ? j1 : mid1;
        CALL(hipEventRecord(b0, s0));
        CALL(hipEventRecord(b1, s1));
        CALL(hipStreamWaitEvent(s0, b1, 0));
        CALL(hipStreamWaitEvent(s1, b0, 0));
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s0, d + 128, 2.f);
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s1, d + 192, 2.f);
        for (int k = 0; mode >= 12 && k < 6; ++k) {
            ba.p = d + 128;
            hipLaunchKernelGGL(k_big, dim3(4), dim3(64), 0, s0, ba);
            ba.p = d + 192;
            hipLaunchKernelGGL(k_big, dim3(4), dim3(64), 0, s1, ba);
        }
    }
    if (mode == 6) {
        CALL(hipEventRecord(mid0, s0));
        CALL(hipStreamWaitEvent(other, mid0, 0));  // uncaptured stream on a captured event
        status("other", other);
    }
    CALL(hipEventRecord(j0, s0));
    CALL(hipStreamWaitEvent(cap, j0, 0));
    if (mode == 7) {  // s1 -> s0 (before s0's join record above is replaced by a later one)
        CALL(hipEventRecord(j1, s1));
        CALL(hipStreamWaitEvent(s0, j1, 0));
        CALL(hipEventRecord(j0, s0));
        CALL(hipStreamWaitEvent(cap, j0, 0));
    }
    if (mode != 3 && mode != 5 && mode != 7 && mode != 8 && mode != 9) {
        CALL(hipEventRecord(j1, s1));
        CALL(hipStreamWaitEvent(cap, j1, 0));
    }
    if (mode == 4) CALL(hipEventRecord(mid1, s1));  // re-record after the join
    hipGraph_t g = nullptr;
    CALL(hipStreamEndCapture(cap, &g));
    std::printf("  graph %p\n", (void*)g);
    std::fflush(stdout);
    status("s1 after", s1);
    if (mode == 8) {
        CALL(hipGraphDestroy(g));
        std::printf("mode 8 done\n");
        return 0;
    }
    if (mode == 9) {
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s1, d, 1.f);
        CALL(hipGetLastError());
        CALL(hipStreamSynchronize(s1));
        std::printf("mode 9 done\n");
        return 0;
    }
    if (mode == 5) {  // the failed EndCapture's handle is not used
        std::printf("mode 5 done\n");
        return 0;
    }
    if (g) {
        hipGraphExec_t x = nullptr;
        CALL(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        if (x) {
            CALL(hipGraphLaunch(x, cap));
            CALL(hipStreamSynchronize(cap));
            hipGraphExecDestroy(x);
        }
        hipGraphDestroy(g);
    }
    CALL(hipDeviceSynchronize());
    float h[256];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    std::printf("  d[0] %.0f d[64] %.0f d[128] %.0f d[192] %.0f\n", h[0], h[64], h[128], h[192]);
    std::printf("mode %d done\n", mode);
    return 0;
}
