// thread_exit_probe.hip -- does a host thread that used HIP and then exited
// break a later multi-stream graph launch (HIP 7.2)? The host-frame path's
// download thread (dis_runtime.hip HostPipe) exits when its context is
// destroyed; a later context's first graph launch crashed the host in the r06
// GPU suite. One mode per process:
//   thread_exit_probe <mode>
//   0  no extra thread, then capture + launch a 3-branch fork/join graph
//   1  a thread calls hipSetDevice and exits (joined) first
//   2  a thread creates a stream, does a pageable D2H on it, destroys the
//      stream and exits (joined) first
//   3  as 2, but the thread stays alive (parked) until after the launch
//   4  as 2, twice, with a graph launch in between
// Prints each step; a host crash shows as the process's signal.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

__global__ void k_add(float* p, float v) { p[threadIdx.x] += v; }

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        std::printf("  %-58s -> %s\n", #x, hipGetErrorName(e_));                  \
        std::fflush(stdout);                                                      \
        if (e_ != hipSuccess) return 1;                                           \
    } while (0)

static void worker(float* d, std::vector<float>* host, bool park, std::mutex* mu, std::condition_variable* cv,
                   bool* release)
{
    hipSetDevice(0);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipMemcpyAsync(host->data(), d, host->size() * sizeof(float), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    hipStreamDestroy(s);
    std::printf("  worker copied\n");
    std::fflush(stdout);
    if (park) {
        std::unique_lock<std::mutex> l(*mu);
        cv->wait(l, [&] { return *release; });
    }
}

static int graph_once(float* d)
{
    hipStream_t cap, own, sub[3];
    hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&own, hipStreamNonBlocking);
    for (auto& x : sub) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    hipEvent_t fork, join[3];
    hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    for (auto& e : join) hipEventCreateWithFlags(&e, hipEventDisableTiming);
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, cap));
    for (int k = 0; k < 3; ++k) {
        CK(hipStreamWaitEvent(sub[k], fork, 0));
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, sub[k], d + 64 * k, 1.f);
    }
    for (int k = 0; k < 3; ++k) {
        CK(hipEventRecord(join[k], sub[k]));
        CK(hipStreamWaitEvent(cap, join[k], 0));
    }
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(cap, &g));
    hipGraphExec_t x = nullptr;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, own));
    CK(hipStreamSynchronize(own));
    hipGraphExecDestroy(x);
    hipGraphDestroy(g);
    return 0;
}

int main(int argc, char** argv)
{
    const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
    std::printf("mode %d\n", mode);
    CK(hipSetDevice(0));
    float* d = nullptr;
    CK(hipMalloc(&d, 1 << 24));
    CK(hipMemset(d, 0, 1 << 24));
    std::vector<float> host(1 << 22);
    std::mutex mu;
    std::condition_variable cv;
    bool release = false;
    std::thread parked;
    if (mode == 1) {
        std::thread t([] { hipSetDevice(0); });
        t.join();
        std::printf("  thread (hipSetDevice only) joined\n");
    } else if (mode == 2 || mode == 4) {
        std::thread t(worker, d, &host, false, &mu, &cv, &release);
        t.join();
        std::printf("  thread joined\n");
    } else if (mode == 3) {
        parked = std::thread(worker, d, &host, true, &mu, &cv, &release);
    }
    if (mode == 3) {
        // let the worker finish its copy before the capture
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
    }
    if (graph_once(d)) return 1;
    if (mode == 4) {
        std::thread t(worker, d, &host, false, &mu, &cv, &release);
        t.join();
        std::printf("  second thread joined\n");
        if (graph_once(d)) return 1;
    }
    if (mode == 3) {
        {
            std::lock_guard<std::mutex> l(mu);
            release = true;
        }
        cv.notify_all();
        parked.join();
    }
    std::printf("mode %d done\n", mode);
    return 0;
}
