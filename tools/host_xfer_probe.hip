// host_xfer_probe.hip -- what the host-frame path can use to move frames and
// flows between pageable caller memory and the device (dis_runtime.hip
// calc_host): is a pageable hipMemcpyAsync asynchronous for the host thread,
// what does registering the caller's buffer cost, how fast does the CPU read
// page-locked staging (default vs non-coherent allocation). One line per test.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("%s -> %s\n", #x, hipGetErrorName(e_));                       \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main()
{
    const size_t flow = 1920ull * 1080 * 8;  // one 1080p flow
    const size_t big = 4 * flow;             // a 4-pair chunk
    const size_t all = 32 * flow;            // a 32-pair batch
    void *d = nullptr, *pin = nullptr, *pin_nc = nullptr;
    CK(hipMalloc(&d, all));
    CK(hipMemset(d, 1, all));
    std::vector<char> host(all, 2);  // pageable, touched
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    // 1. pageable D2H of one chunk: host time in the call vs to completion
    for (int rep = 0; rep < 3; ++rep) {
        const double t0 = now();
        CK(hipMemcpyAsync(host.data(), d, big, hipMemcpyDeviceToHost, s));
        const double t1 = now();
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        std::printf("pageable D2H %zu MB: call returns after %.3f ms, done after %.3f ms (%.1f GB/s)\n", big >> 20,
                    (t1 - t0) * 1e3, (t2 - t0) * 1e3, big / (t2 - t0) / 1e9);
    }
    for (int rep = 0; rep < 2; ++rep) {
        const double t0 = now();
        CK(hipMemcpyAsync(d, host.data(), big, hipMemcpyHostToDevice, s));
        const double t1 = now();
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        std::printf("pageable H2D %zu MB: call returns after %.3f ms, done after %.3f ms (%.1f GB/s)\n", big >> 20,
                    (t1 - t0) * 1e3, (t2 - t0) * 1e3, big / (t2 - t0) / 1e9);
    }
    // 2. a pageable D2H queued behind 2 ms of device work: does the call wait?
    {
        CK(hipMemsetAsync(d, 3, all, s));
        CK(hipMemsetAsync(d, 4, all, s));
        const double t0 = now();
        CK(hipMemcpyAsync(host.data(), d, big, hipMemcpyDeviceToHost, s));
        const double t1 = now();
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        std::printf("pageable D2H behind queued work: call returns after %.3f ms, done after %.3f ms\n",
                    (t1 - t0) * 1e3, (t2 - t0) * 1e3);
    }
    // 3. register / unregister the caller's buffer
    for (size_t sz : {big, all}) {
        const double t0 = now();
        CK(hipHostRegister(host.data(), sz, hipHostRegisterDefault));
        const double t1 = now();
        CK(hipMemcpyAsync(host.data(), d, sz, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        const double t2 = now();
        CK(hipHostUnregister(host.data()));
        const double t3 = now();
        std::printf("register %zu MB %.3f ms, D2H %.3f ms (%.1f GB/s), unregister %.3f ms\n", sz >> 20,
                    (t1 - t0) * 1e3, (t2 - t1) * 1e3, sz / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
    }
    // 4. CPU reads of page-locked staging: default vs non-coherent
    CK(hipHostMalloc(&pin, big, hipHostMallocDefault));
    CK(hipHostMalloc(&pin_nc, big, hipHostMallocNonCoherent));
    for (int k = 0; k < 2; ++k) {
        void* p = k ? pin_nc : pin;
        CK(hipMemcpyAsync(p, d, big, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        for (int nt : {1, 4}) {
            const double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    const size_t a = big * t / nt, b = big * (t + 1) / nt;
                    std::memcpy(host.data() + a, static_cast<char*>(p) + a, b - a);
                });
            for (auto& x : th) x.join();
            const double t1 = now();
            std::printf("CPU copy out of %s staging, %d thread(s): %.1f GB/s\n", k ? "non-coherent" : "default",
                        nt, big / (t1 - t0) / 1e9);
        }
        const double t0 = now();
        CK(hipMemcpyAsync(p, d, big, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        std::printf("D2H into %s staging: %.1f GB/s\n", k ? "non-coherent" : "default", big / (now() - t0) / 1e9);
    }
    // 5. plain CPU copy pageable -> pageable
    {
        std::vector<char> other(big, 5);
        const double t0 = now();
        std::memcpy(other.data(), host.data(), big);
        std::printf("CPU copy pageable -> pageable, 1 thread: %.1f GB/s\n", big / (now() - t0) / 1e9);
    }
    hipHostFree(pin);
    hipHostFree(pin_nc);
    hipFree(d);
    std::printf("done\n");
    return 0;
}
