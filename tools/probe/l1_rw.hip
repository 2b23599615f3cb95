// Developer probe (GPU box): does a wave read back, from another lane, global data it wrote after
// a __syncthreads(), when the old lines were in the vector L1?  u16 / u32 / f64 stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define AS __attribute__((address_space(1)))
template <class T>
__global__ __launch_bounds__(64) void probe(T *buf_, int n, int rounds, unsigned long long *bad) {
    AS T *buf = (AS T *)(buf_ + (size_t)blockIdx.x * n);
    const int l = threadIdx.x;
    unsigned long long nb = 0;
    for (int r = 1; r <= rounds; ++r) {
        T acc = 0;
        for (int i = l; i < n; i += 64) acc += buf[i];          // old lines into L1
        if (acc == (T)12345) buf[0] = 0;                      // keep the loads
        __syncthreads();
        for (int i = l; i < n; i += 64) buf[(i * 7 + 3) % n] = (T)(r * 31 + (i * 7 + 3) % n);  // rewrite
        __syncthreads();
        for (int i = l; i < n; i += 64) {                      // read back (other lanes' writes)
            const int j = (i * 13 + 5) % n;
            if (buf[j] != (T)(r * 31 + j)) ++nb;
        }
        __syncthreads();
    }
    if (nb) atomicAdd(bad, nb);
}
template <class T>
void run(const char *name) {
    const int n = 1024, blocks = 1024, rounds = 50;
    T *d; unsigned long long *bad, h = 0;
    hipMalloc(&d, sizeof(T) * n * blocks); hipMemset(d, 0, sizeof(T) * n * blocks);
    hipMalloc(&bad, 8); hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(probe<T>, dim3(blocks), dim3(64), 0, 0, d, n, rounds, bad);
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    printf("%s: stale reads %llu of %llu\n", name, h, (unsigned long long)n * blocks * rounds);
    hipFree(d); hipFree(bad);
}
int main() {
    run<uint16_t>("u16");
    run<uint32_t>("u32");
    run<double>("f64");
    return 0;
}
