// valu_rate.hip — issue rate of scalar vs packed fp32 VALU ops on gfx950:
// chains of independent v_fma_f32 / v_pk_fma_f32 / v_pk_add_f32 per lane, at
// 1..8 waves per SIMD; prints wave-instructions per SIMD per ns and the
// implied cycles per wave-instruction at the measured kernel clock.
//   hipcc --offload-arch=gfx950 -O3 scripts/valu_rate.hip -o scripts/bin/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096, CH = 8;

template <int OP>
__global__ __launch_bounds__(256) void k(float *out, float c)
{
    f2 v[CH];
    for (int i = 0; i < CH; ++i) v[i] = (f2){(float)threadIdx.x + i, (float)i};
    const f2 cc = (f2){c, c};
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if (OP == 0) {
                asm volatile("v_fma_f32 %0, %1, %0, %1" : "+v"(v[i].x) : "v"(cc.x));
                asm volatile("v_fma_f32 %0, %1, %0, %1" : "+v"(v[i].y) : "v"(cc.x));
            } else if (OP == 1) {
                asm volatile("v_pk_fma_f32 %0, %1, %0, %1" : "+v"(v[i]) : "v"(cc));
            } else if (OP == 2) {
                asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(v[i]) : "v"(cc));
            } else {
                asm volatile("v_add_f32 %0, %1, %0" : "+v"(v[i].x) : "v"(cc.x));
                asm volatile("v_add_f32 %0, %1, %0" : "+v"(v[i].y) : "v"(cc.x));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < CH; ++i) s += v[i].x + v[i].y;
    if (s == 1.2345f) out[0] = s;
}

int main()
{
    float *o;
    (void)hipMalloc(&o, 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *names[] = {"v_fma_f32 x2", "v_pk_fma_f32", "v_pk_add_f32", "v_add_f32 x2"};
    for (int op = 0; op < 4; ++op)
        for (int wps : {1, 2, 4, 8}) {
            // 256 CUs x 4 SIMDs x wps waves: blocks of 4 waves, one per SIMD
            const int blocks = 256 * wps;
            auto f = op == 0 ? k<0> : op == 1 ? k<1> : op == 2 ? k<2> : k<3>;
            for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, o, 0.999f);
            (void)hipEventRecord(a);
            for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, o, 0.999f);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const double insts = (op == 1 || op == 2 ? 1.0 : 2.0) * CH * ITER * 5.0 * wps;  // per SIMD
            const double ns = ms * 1e6;
            std::printf("%-14s %d waves/SIMD: %.3f wave-inst/ns/SIMD -> %.2f cyc/inst at 2.4 GHz, %.1f TFLOP/s\n",
                        names[op], wps, insts / ns, 2.4 * ns / insts,
                        (op < 2 ? 2.0 : 1.0) * 64 * 2 * CH * ITER * 5.0 * wps * 1024 / ns / 1e3);
        }
    return 0;
}
