// pcie_probe.hip — host<->device copy ceilings on this MI355X box.
//
// What the host-array drop-in path can reach at best: pinned (hipHostMalloc)
// and pageable (malloc) sources, one and two streams, several chunk sizes;
// plus the device->host direction for the icons.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pcie_probe.hip -o tools/pcie_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t total = 1ull << 30;  // 1 GiB per measurement
    void* dev;
    CK(hipMalloc(&dev, total));
    void* pinned;
    CK(hipHostMalloc(&pinned, total, hipHostMallocDefault));
    memset(pinned, 1, total);
    void* pageable = malloc(total);
    memset(pageable, 1, total);
    hipStream_t s[4];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));

    for (int src_kind = 0; src_kind < 2; ++src_kind) {
        const char* name = src_kind ? "pageable" : "pinned";
        void* host = src_kind ? pageable : pinned;
        for (size_t chunk : {(size_t)4 << 20, (size_t)16 << 20, (size_t)64 << 20, (size_t)256 << 20}) {
            for (int ns : {1, 2, 4}) {
                CK(hipDeviceSynchronize());
                double best = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    double t0 = now();
                    size_t k = 0;
                    for (size_t off = 0; off < total; off += chunk, ++k)
                        CK(hipMemcpyAsync((char*)dev + off, (char*)host + off, chunk,
                                          hipMemcpyHostToDevice, s[k % ns]));
                    for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(s[i]));
                    double gbs = total / (now() - t0) / 1e9;
                    best = gbs > best ? gbs : best;
                }
                printf("h2d src=%s chunk=%zuMiB streams=%d  %.1f GB/s\n", name, chunk >> 20, ns, best);
            }
        }
        // the same bytes issued from several host threads (one stream each)
        for (int nt : {2, 4, 8}) {
            double best = 0;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipDeviceSynchronize());
                double t0 = now();
                std::vector<std::thread> th;
                const size_t per = total / nt;
                for (int t = 0; t < nt; ++t)
                    th.emplace_back([&, t] {
                        hipStream_t st;
                        (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
                        (void)hipMemcpyAsync((char*)dev + t * per, (char*)host + t * per, per,
                                             hipMemcpyHostToDevice, st);
                        (void)hipStreamSynchronize(st);
                        (void)hipStreamDestroy(st);
                    });
                for (auto& x : th) x.join();
                double gbs = total / (now() - t0) / 1e9;
                best = gbs > best ? gbs : best;
            }
            printf("h2d src=%s threads=%d  %.1f GB/s\n", name, nt, best);
        }
    }
    for (size_t chunk : {(size_t)16 << 20, (size_t)256 << 20}) {
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            double t0 = now();
            for (size_t off = 0; off < total; off += chunk)
                CK(hipMemcpyAsync((char*)pinned + off, (char*)dev + off, chunk, hipMemcpyDeviceToHost, s[0]));
            CK(hipStreamSynchronize(s[0]));
            double gbs = total / (now() - t0) / 1e9;
            best = gbs > best ? gbs : best;
        }
        printf("d2h dst=pinned chunk=%zuMiB  %.1f GB/s\n", chunk >> 20, best);
    }
    // host memcpy bandwidth (pageable -> pinned), 1..8 threads: the CPU side of a staged upload
    for (int nt : {1, 2, 4, 8}) {
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            double t0 = now();
            std::vector<std::thread> th;
            const size_t per = total / nt;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] { memcpy((char*)pinned + t * per, (char*)pageable + t * per, per); });
            for (auto& x : th) x.join();
            double gbs = total / (now() - t0) / 1e9;
            best = gbs > best ? gbs : best;
        }
        printf("host memcpy pageable->pinned threads=%d  %.1f GB/s\n", nt, best);
    }
    return 0;
}
