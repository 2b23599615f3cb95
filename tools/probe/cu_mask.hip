// Developer probe (GPU box): where do the workgroups of a CU-masked stream run?  For each mask
// layout, a kernel of many short workgroups is launched on a stream created with
// hipExtStreamCreateWithCUMask and every workgroup records its hardware ids (XCC, shader engine,
// CU); the program prints how many distinct (xcc, se, cu) triples each XCC saw.  Answers how the
// driver maps CU-mask bits to XCDs on gfx950 (the ccdgpu_init_copy_cus reservation).
//
//   hipcc --offload-arch=gfx950 -O2 tools/probe/cu_mask.hip -o tools/probe/cu_mask && tools/probe/cu_mask
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

// s_getreg operand: (size - 1) << 11 | offset << 6 | register id; HW_ID = 4, XCC_ID = 20 (gfx940+)
__global__ void whereami(uint32_t *out, int spin) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

static void run(const char *tag, int n_cu, const std::vector<uint32_t> &mask) {
    hipStream_t s;
    if (mask.empty()) {
        if (hipStreamCreate(&s) != hipSuccess) return;
    } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        std::printf("%s: stream create failed\n", tag);
        return;
    }
    const int blocks = 4096;
    uint32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t) * 2 * blocks) != hipSuccess) return;
    hipLaunchKernelGGL(whereami, dim3(blocks), dim3(64), 0, s, d, 20000);
    std::vector<uint32_t> h(2 * blocks);
    (void)hipMemcpyAsync(h.data(), d, sizeof(uint32_t) * 2 * blocks, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    std::map<int, std::set<int>> per_xcc;  // xcc -> {se * 64 + sh * 16 + cu}
    for (int b = 0; b < blocks; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        per_xcc[(int)xcc].insert(se * 64 + sh * 16 + cu);
    }
    int total = 0;
    std::string line;
    for (auto &kv : per_xcc) {
        total += (int)kv.second.size();
        line += " xcc" + std::to_string(kv.first) + ":" + std::to_string(kv.second.size());
    }
    std::printf("%-28s CUs used %3d of %d |%s\n", tag, total, n_cu, line.c_str());
    if (per_xcc.count(7) && per_xcc[7].size() <= 8) {
        std::printf("    xcc7 CUs (se*64+sh*16+cu):");
        for (int v : per_xcc[7]) std::printf(" %d", v);
        std::printf("\n");
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int n = p.multiProcessorCount, nw = (n + 31) / 32, per = n / 8;
    std::printf("%s, %d CUs\n", p.gcnArchName, n);
    auto make = [&](auto pred) {
        std::vector<uint32_t> m(nw, 0u);
        for (int cu = 0; cu < n; ++cu)
            if (pred(cu)) m[cu / 32] |= 1u << (cu % 32);
        return m;
    };
    run("unmasked", n, {});
    run("blocked reserved (r3-r4)", n, make([&](int cu) { return cu % per == per - 1; }));
    run("blocked detection", n, make([&](int cu) { return cu % per != per - 1; }));
    run("interleaved reserved", n, make([&](int cu) { return cu >= n - 8; }));
    run("interleaved detection", n, make([&](int cu) { return cu < n - 8; }));
    run("bits 0-7", n, make([&](int cu) { return cu < 8; }));
    run("bits 0-31", n, make([&](int cu) { return cu < 32; }));
    return 0;
}
