// Correctness probe (round 3): a v_pk_fma_f32 result read by v_mov_b32_dpp (wave_shl:1 /
// wave_shr:1) after K independent filler instructions (VALU or SALU) or an s_nop, all in one
// asm block (the compiler's hazard recognizer is out of the picture).  Prints the number of
// wrong lanes per case: the distance asm-produced packed results need before a DPP read.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

// MODE 0: K VALU fillers; 1: K SALU fillers; 2: s_nop K-1; HI: read the high half
#define HZ_PRE "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n s_nop 4\n v_pk_fma_f32 v[40:41], %3, %4, v[40:41] op_sel_hi:[0,1,1]\n"
#define HZ_POST ".if %7\n v_mov_b32_dpp %0, v41 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
                ".else\n v_mov_b32_dpp %0, v40 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n .endif\n"
template <int MODE, int K, int HI>
__global__ void k(const float* in, float* out) {
    const int l = threadIdx.x;
    f2 a = {in[l], in[64 + l]}, w = {2.0f, 0.5f};
    float c0 = in[128 + l], c1 = in[192 + l];
    float t = in[l] * 3.0f, r;
    int s = blockIdx.x;
    asm volatile("" : "+v"(w), "+v"(t));
    if constexpr (MODE == 0)
        asm volatile(HZ_PRE
            ".if %6 >= 1\n v_add_f32 %5, 1.0, %5\n .endif\n"
            ".if %6 >= 2\n v_add_f32 %5, 1.0, %5\n .endif\n"
            ".if %6 >= 3\n v_add_f32 %5, 1.0, %5\n .endif\n"
            ".if %6 >= 4\n v_add_f32 %5, 1.0, %5\n .endif\n" HZ_POST
            : "=&v"(r) : "v"(c0), "v"(c1), "v"(w), "v"(a), "v"(t), "n"(K), "n"(HI) : "v40", "v41");
    else if constexpr (MODE == 1)
        asm volatile(HZ_PRE
            ".if %6 >= 1\n s_add_u32 %5, %5, 1\n .endif\n"
            ".if %6 >= 2\n s_add_u32 %5, %5, 1\n .endif\n"
            ".if %6 >= 3\n s_add_u32 %5, %5, 1\n .endif\n"
            ".if %6 >= 4\n s_add_u32 %5, %5, 1\n .endif\n" HZ_POST
            : "=&v"(r) : "v"(c0), "v"(c1), "v"(w), "v"(a), "s"(s), "n"(K), "n"(HI) : "v40", "v41", "scc");
    else
        asm volatile(HZ_PRE
            ".if %6 >= 1\n s_nop %6 - 1\n .endif\n" HZ_POST
            : "=&v"(r) : "v"(c0), "v"(c1), "v"(w), "v"(a), "v"(t), "n"(K), "n"(HI) : "v40", "v41");
    out[l] = r;
}

template <int MODE, int K, int HI>
void run(float* din, float* dout, const std::vector<float>& hin) {
    hipLaunchKernelGGL((k<MODE, K, HI>), dim3(1), dim3(64), 0, 0, din, dout);
    CK(hipDeviceSynchronize());
    std::vector<float> o(64);
    CK(hipMemcpy(o.data(), dout, 256, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int src = l + 1;
        float e = 0.f;
        if (src < 64) e = HI ? hin[192 + src] + 2.0f * hin[64 + src] : hin[128 + src] + 2.0f * hin[src];
        if (o[l] != e) ++bad;
    }
    const char* m = MODE == 0 ? "VALU" : (MODE == 1 ? "SALU" : "s_nop");
    printf("pk_fma -> %d %-5s -> dpp (%s half): %2d of 64 lanes wrong\n", K, m, HI ? "hi" : "lo", bad);
}


// DPP -> pk_fma: v40 = dpp(x) wave_shr:1, v41 = y; K fillers; pk_fma v[42:43] = w.lo * v[40:41] + c
template <int MODE, int K>
__global__ void k2(const float* in, float* out) {
    const int l = threadIdx.x;
    float x = in[l], y = in[64 + l], c0 = in[128 + l], c1 = in[192 + l], t = in[l] * 3.0f;
    f2 w = {2.0f, 0.5f};
    float r0, r1;
    int s = blockIdx.x;
    asm volatile("" : "+v"(w), "+v"(t));
    if constexpr (MODE == 0)
        asm volatile(
            "v_mov_b32 v41, %3\n v_mov_b32 v42, %4\n v_mov_b32 v43, %5\n s_nop 4\n"
            "v_mov_b32_dpp v40, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            ".if %8 >= 1\n v_add_f32 %7, 1.0, %7\n .endif\n"
            ".if %8 >= 2\n v_add_f32 %7, 1.0, %7\n .endif\n"
            ".if %8 >= 3\n v_add_f32 %7, 1.0, %7\n .endif\n"
            "v_pk_fma_f32 v[42:43], %6, v[40:41], v[42:43] op_sel_hi:[0,1,1]\n"
            "s_nop 4\n v_mov_b32 %0, v42\n v_mov_b32 %1, v43\n"
            : "=&v"(r0), "=&v"(r1) : "v"(x), "v"(y), "v"(c0), "v"(c1), "v"(w), "v"(t), "n"(K)
            : "v40", "v41", "v42", "v43");
    else
        asm volatile(
            "v_mov_b32 v41, %3\n v_mov_b32 v42, %4\n v_mov_b32 v43, %5\n s_nop 4\n"
            "v_mov_b32_dpp v40, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            ".if %8 >= 1\n s_nop %8 - 1\n .endif\n"
            "v_pk_fma_f32 v[42:43], %6, v[40:41], v[42:43] op_sel_hi:[0,1,1]\n"
            "s_nop 4\n v_mov_b32 %0, v42\n v_mov_b32 %1, v43\n"
            : "=&v"(r0), "=&v"(r1) : "v"(x), "v"(y), "v"(c0), "v"(c1), "v"(w), "v"(t), "n"(K)
            : "v40", "v41", "v42", "v43");
    out[l] = r0;
    out[64 + l] = r1;
}

template <int MODE, int K>
void run2(float* din, float* dout, const std::vector<float>& hin) {
    hipLaunchKernelGGL((k2<MODE, K>), dim3(1), dim3(64), 0, 0, din, dout);
    CK(hipDeviceSynchronize());
    std::vector<float> o(128);
    CK(hipMemcpy(o.data(), dout, 512, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const float px = l ? hin[l - 1] : 0.f;
        if (o[l] != hin[128 + l] + 2.0f * px || o[64 + l] != hin[192 + l] + 2.0f * hin[64 + l]) ++bad;
    }
    printf("dpp -> %d %-5s -> pk_fma: %2d of 64 lanes wrong\n", K, MODE ? "s_nop" : "VALU", bad);
}

// operand-form probe: d = w[lo] * a + c[lo] (op_sel_hi:[0,1,0]) with w an SGPR pair (SRC 1)
// or a VGPR pair (SRC 0); also the other op_sel forms the fused kernel uses
template <int SRC, int FORM>
__global__ void k3(const float* in, float* out, f2 ws) {
    const int l = threadIdx.x;
    f2 a = {in[l], in[64 + l]}, c = {in[128 + l], in[192 + l]}, d;
    f2 wv = ws;
    asm volatile("" : "+v"(wv));
#define K3(SEL) if constexpr (SRC) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 " SEL : "=v"(d) : "s"(ws), "v"(a), "v"(c)); \
                else asm volatile("v_pk_fma_f32 %0, %1, %2, %3 " SEL : "=v"(d) : "v"(wv), "v"(a), "v"(c));
    if constexpr (FORM == 0) { K3("op_sel_hi:[0,1,0]") }
    if constexpr (FORM == 1) { K3("op_sel_hi:[0,1,1]") }
    if constexpr (FORM == 2) { K3("op_sel:[1,0,0] op_sel_hi:[1,1,1]") }
    if constexpr (FORM == 3) { K3("op_sel:[1,0,1] op_sel_hi:[1,1,1]") }
    if constexpr (FORM == 4) { K3("op_sel:[1,0,0] op_sel_hi:[1,1,0]") }
    if constexpr (FORM == 5) { K3("op_sel:[0,0,1] op_sel_hi:[0,1,1]") }
    out[l] = d.x;
    out[64 + l] = d.y;
}

template <int SRC, int FORM>
void run3(float* din, float* dout, const std::vector<float>& hin) {
    const float w0 = 2.0f, w1 = 0.5f;
    hipLaunchKernelGGL((k3<SRC, FORM>), dim3(1), dim3(64), 0, 0, din, dout, f2{w0, w1});
    CK(hipDeviceSynchronize());
    std::vector<float> o(128);
    CK(hipMemcpy(o.data(), dout, 512, hipMemcpyDeviceToHost));
    // expected per form: (w for lo, w for hi, c for lo, c for hi)
    const float WL[6] = {w0, w0, w1, w1, w1, w0}, WH[6] = {w0, w0, w1, w1, w1, w0};
    const int CL[6] = {0, 0, 0, 1, 0, 1}, CH[6] = {0, 1, 1, 1, 0, 1};
    int bad = 0, l0 = -1;
    float g0 = 0, g1 = 0;
    for (int l = 0; l < 64; ++l) {
        const float e0 = WL[FORM] * hin[l] + hin[128 + 64 * CL[FORM] + l];
        const float e1 = WH[FORM] * hin[64 + l] + hin[128 + 64 * CH[FORM] + l];
        if (o[l] != e0 || o[64 + l] != e1) { if (l0 < 0) { l0 = l; g0 = o[l]; g1 = o[64 + l]; } ++bad; }
    }
    printf("pk_fma form %d, weight in %s: %2d of 64 lanes wrong", FORM, SRC ? "SGPR" : "VGPR", bad);
    if (l0 >= 0) printf("  (lane %d got %g %g)", l0, g0, g1);
    printf("\n");
}

int main() {
    float *din, *dout;
    CK(hipMalloc(&din, 1024)); CK(hipMalloc(&dout, 512));
    std::vector<float> hin(256);
    for (int i = 0; i < 256; ++i) hin[i] = 1.0f + 0.125f * i;
    CK(hipMemcpy(din, hin.data(), 1024, hipMemcpyHostToDevice));
    run<0, 0, 0>(din, dout, hin); run<0, 1, 0>(din, dout, hin); run<0, 2, 0>(din, dout, hin);
    run<0, 3, 0>(din, dout, hin); run<0, 4, 0>(din, dout, hin);
    run<0, 0, 1>(din, dout, hin); run<0, 1, 1>(din, dout, hin); run<0, 2, 1>(din, dout, hin);
    run<0, 3, 1>(din, dout, hin); run<0, 4, 1>(din, dout, hin);
    run<1, 1, 0>(din, dout, hin); run<1, 2, 0>(din, dout, hin); run<1, 3, 1>(din, dout, hin);
    run<2, 1, 0>(din, dout, hin); run<2, 2, 0>(din, dout, hin); run<2, 3, 1>(din, dout, hin);
    run<2, 4, 1>(din, dout, hin);
    run2<0, 0>(din, dout, hin); run2<0, 1>(din, dout, hin); run2<0, 2>(din, dout, hin);
    run2<0, 3>(din, dout, hin); run2<1, 1>(din, dout, hin); run2<1, 2>(din, dout, hin);
    run3<0, 0>(din, dout, hin); run3<1, 0>(din, dout, hin); run3<0, 1>(din, dout, hin); run3<1, 1>(din, dout, hin);
    run3<0, 2>(din, dout, hin); run3<1, 2>(din, dout, hin); run3<0, 3>(din, dout, hin); run3<1, 3>(din, dout, hin);
    run3<0, 4>(din, dout, hin); run3<1, 4>(din, dout, hin); run3<0, 5>(din, dout, hin); run3<1, 5>(din, dout, hin);
    return 0;
}
