#include <hip/hip_runtime.h>
__device__ __attribute__((always_inline)) inline float sh_bcast(float c, const float (&bs)[16]) {
    float a;
    asm("s_nop 1\n\t"
        "v_mov_b32_dpp %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %4 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %7 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %10 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %11 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %13 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %14 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %15 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %1, %16 row_newbcast:15 row_mask:0xf bank_mask:0xf"
        : "=&v"(a)
        : "v"(c), "v"(bs[1]), "v"(bs[2]), "v"(bs[3]), "v"(bs[4]), "v"(bs[5]), "v"(bs[6]), "v"(bs[7]), "v"(bs[8]),
          "v"(bs[9]), "v"(bs[10]), "v"(bs[11]), "v"(bs[12]), "v"(bs[13]), "v"(bs[14]), "v"(bs[15]));
    return a;
}
__global__ void k(const float* __restrict__ sh, const float* __restrict__ bsin, float* out, float* ref) {
    __shared__ float s[48];
    const int l = threadIdx.x;
    if (l < 48) s[l] = sh[l];
    __syncthreads();
    float bs[16];
    for (int q = 0; q < 16; ++q) bs[q] = bsin[q * 64 + l];
    for (int ch = 0; ch < 3; ++ch) {
        const float a = sh_bcast(s[ch * 16 + (l & 15)], bs);
        out[ch * 64 + l] = a;
        float r = s[ch * 16];
        for (int q = 1; q < 16; ++q) r = fmaf(bs[q], s[ch * 16 + q], r);
        ref[ch * 64 + l] = r;
    }
}
int main() {
    float *sh, *bs, *o, *r;
    hipMallocManaged(&sh, 48 * 4); hipMallocManaged(&bs, 16 * 64 * 4); hipMallocManaged(&o, 192 * 4); hipMallocManaged(&r, 192 * 4);
    for (int i = 0; i < 48; ++i) sh[i] = 0.37f * i - 3.1f + 1e-3f * i * i;
    for (int i = 0; i < 1024; ++i) bs[i] = 0.013f * (i % 97) - 0.5f;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, sh, bs, o, r);
    hipDeviceSynchronize();
    int bad = 0;
    for (int i = 0; i < 192; ++i) bad += __builtin_bit_cast(unsigned, o[i]) != __builtin_bit_cast(unsigned, r[i]);
    printf("mismatches %d  o[5]=%g r[5]=%g o[130]=%g r[130]=%g\n", bad, o[5], r[5], o[130], r[130]);
    return bad != 0;
}
