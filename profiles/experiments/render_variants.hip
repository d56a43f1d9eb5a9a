// render_variants.hip -- measured experiment variants of the COR shading loop and the footprint test, moved out
// of the product source (3dgs-raytrace_amd/csrc/gsrt_render.hip) in round 2. NOT built; kept as the record of
// what was tried. They were compiled in the product file behind -DGSRT_MFMA_SH=1, -DGSRT_DPP_SH=1,
// -DGSRT_X_OBB, -DGSRT_X_SLABFREE (last commit with them in place: 103b185). Results (C3, one MI355X):
//   GSRT_MFMA_SH    SH-3 colours on v_mfma_f32_16x16x4f32: bit-exact, render kernel 1.46 -> 1.96 ms
//   GSRT_DPP_SH     SH coefficients broadcast by DPP row_newbcast: bit-exact, 1.42 -> 1.60 ms
//   GSRT_X_OBB      oriented-box footprint test instead of the exact ellipse-rectangle test: more candidates
//   GSRT_X_SLABFREE per-tile slab-free flags: render -1 %, group lists +20 %, net loss
// See DESIGN.md §3 "Measured dead ends".

// ---- GSRT_X_OBB (footprint slabs)
#ifdef GSRT_X_OBB  // experiment build: the previous oriented-box test (two slabs across the ellipse's axes)
__device__ inline bool slab_meets(const float4 e, float cx, float cy, float hw, float hh) {
    return fabsf(fmaf(e.x, cx, fmaf(e.y, cy, -e.z))) <= fmaf(fabsf(e.x), hw, fmaf(fabsf(e.y), hh, 1.0f));
}
#endif

// ---- GSRT_MFMA_SH
// ---- SH-3 colours on MFMA (k_render_cor with SH, production path)
//
// For the kGroup = 4 candidates of a stage and the 64 rays of the wave, D[n][ray] = sum_k SH[n][k] Y[k][ray]
// with n = 3 c + ch (12 of 16 rows used) and Y the rays' SH basis: per 16-ray tile t four
// v_mfma_f32_16x16x4f32 (K = 4 each, k ascending), whose accumulation is the fmaf chain acc = fma(a_k, b_k, acc)
// bit for bit (profiles/probes/mfma_f32_chain.hip). The oracle's sum s0 y0 + fma chain equals it: only the sign
// of an exact zero can differ, and + 0.5 removes it. Operand layouts (lane l):
//   A[i = n][k]: SH[n = l % 16][k = 4 s + l / 16]  = StageM::shT[l][s] (one ds_read_b128 per stage)
//   B[k][j]:     Y[k = 4 s + l / 16][ray 16 t + l % 16] = CorRay::bs[4 t + s] (per ray, set up once per pass)
//   D:           lane l holds rows n = 4 (l / 16) + r (r = 0..3) of column l % 16 (ray 16 t + l % 16)
// Four 16x16 blocks (lane group g x tile t) are transposed with v_permlane32/16_swap so that every lane holds
// the 16 rows of its own ray (rows 12..15 are padding).
static_assert(kGroup == 4, "the MFMA SH path covers 4 candidates x 3 channels in one 16-row block");
struct StageM {
    SplatRec rec[kGroup];   // 256 B
    float shT[64][4];       // 1 KB: shT[l][s] = SH[n = l % 16][k = 4 s + l / 16], n = 3 c + ch (n >= 12: padding)
};
static_assert(sizeof(StageM) == 1280, "StageM layout");
constexpr uint32_t kStageOpsM = 5;  // DMA instructions per MFMA stage: 1 for the records + 4 SH gathers

// issue the LDS-DMA of stage g0: lanes 0..15 the records (16-B quarters), then four 4-B gathers j = 0..3 in
// which lane i loads SH[n = i / 4][k = 4 (i % 4) + j] of its candidate into shT word 64 j + i.
__device__ inline void stage_issue_m(const uint32_t* ids, uint32_t count, uint32_t g0, uint32_t lane, StageM* dst,
                                    const SplatRec* recs, const float* sh) {
    {
        uint32_t c = g0 + (lane >> 2);
        c = c < count ? c : g0;
        if (lane < 16) {  // lane 0 always issues: every stage is exactly kStageOpsM DMA instructions
            const uint32_t id = ids[c] & kIdMask;
            __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const char*>(recs) + (size_t)id * 64 + (lane & 3) * 16),
                                             (void*)dst->rec, 16, 0, 0);
        }
    }
    const uint32_t n = lane >> 2;
    uint32_t c = g0 + (n < 12 ? n / 3 : 0u);
    c = c < count ? c : g0;
    const uint32_t ch = n < 12 ? n % 3 : 0u;
    const uint32_t id = ids[c] & kIdMask;
    const float* src = sh + (size_t)id * 48 + ch * 16 + (lane & 3) * 4;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(src + j), (void*)(&dst->shT[16 * j][0]), 4, 0, 0);
}

// bs[16] (the lane's own ray's SH basis) -> the MFMA B operands bs[4 t + s] = Y[4 s + l / 16][ray 16 t + l % 16],
// through LDS scratch (>= 16 x 17 floats, padded rows: conflict-free). Every lane of the wave takes part.
__device__ inline void basis_to_mfma(float bs[16], float* scratch, uint32_t lane) {
    float out[16];
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
        __syncthreads();
        if (lane / 16 == t) {
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) scratch[(lane % 16) * 17 + k] = bs[k];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t s4 = 0; s4 < 4; ++s4) out[4 * t + s4] = scratch[(lane % 16) * 17 + 4 * s4 + lane / 16];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) bs[i] = out[i];
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// swap helpers on float bits: permlane32_swap(x, y): x' = [x.lo32, y.lo32], y' = [x.hi32, y.hi32];
// permlane16_swap(x, y): x' = rows [x0, y0, x2, y2], y' = rows [x1, y1, x3, y3] (rows of 16 lanes)
__device__ inline void swap32(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}
__device__ inline void swap16(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}

// ds_read_b128 outside the compiler's view: its waitcnt pass does not tell the stage buffers' LDS-DMAs apart and
// would wait for every one in flight (vmcnt(0)) before this read; the stage's own DMA was waited for (wait()).
__device__ inline f32x4 lds_read_b128_asm(const void* p) {
    f32x4 v;
    const uint32_t a = (uint32_t)(uintptr_t)p;  // LDS offset (the shared aperture is 4-GiB aligned)
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// the stage's SH sums for the lane's own ray: out[n] = sum_k SH[n][k] Y[k] (n = 3 c + ch; out[12..15] padding)
__device__ inline void stage_sh_mfma(const StageM* stg, const float bm[16], uint32_t lane, float out[16]) {
    const f32x4 a4 = lds_read_b128_asm(&stg->shT[lane][0]);
    const float a[4] = {a4[0], a4[1], a4[2], a4[3]};
    f32x4 acc[4];
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (uint32_t s4 = 0; s4 < 4; ++s4)  // K steps outer: the four tiles' chains interleave in the MFMA pipe
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s4], bm[4 * t + s4], acc[t], 0, 0, 0);
    // acc[t] in lane group g = block X[g][t] (rows n = 4 g + r of rays 16 t + l % 16); transpose to X[t][g]
    float v[4][4];
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t)
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) v[t][r] = acc[t][r];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
        swap32(v[0][r], v[2][r]);
        swap32(v[1][r], v[3][r]);
        swap16(v[0][r], v[1][r]);
        swap16(v[2][r], v[3][r]);
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) out[4 * j + r] = v[j][r];
}

// ---- GSRT_DPP_SH
// SH-3 sums of one staged candidate for every lane's ray, a[ch] = s[ch][0] y0 + fma chain over k = 1..15 (the
// oracle's order; fmac's multiply operands commute). The 48 coefficients are not broadcast from LDS (12
// ds_read_b128 of 4 LDS cycles each): lane l holds coefficient k = l % 16 of each channel (cv, 3 ds_read_b32
// issued early by the caller; the four rows of 16 lanes read the same 64 B), and each FMA takes coefficient k
// from lane k of its row with DPP row_newbcast:k. DPP reads other lanes' registers, so the FMAs run as one
// volatile asm with the full wave active (a wave-uniform branch; the blend that uses the sums is masked
// afterwards), and cv must have been loaded with the full wave active too. s_nop 1: the DPP-source hazard.
__device__ inline void sh_dots_dpp(const float cv[3], const float bs[16], float a[3]) {
    asm volatile(
        "s_nop 1\n\t"
        "v_mul_f32_dpp %[a0], %[c0], %[b0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f32_dpp %[a1], %[c1], %[b0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_mul_f32_dpp %[a2], %[c2], %[b0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a0], %[c0], %[b15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a1], %[c1], %[b15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %[a2], %[c2], %[b15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
        : [a0] "=&v"(a[0]), [a1] "=&v"(a[1]), [a2] "=&v"(a[2])
        : [c0] "v"(cv[0]), [c1] "v"(cv[1]), [c2] "v"(cv[2]), [b0] "v"(bs[0]), [b1] "v"(bs[1]), [b2] "v"(bs[2]), [b3] "v"(bs[3]), [b4] "v"(bs[4]), [b5] "v"(bs[5]), [b6] "v"(bs[6]), [b7] "v"(bs[7]), [b8] "v"(bs[8]), [b9] "v"(bs[9]), [b10] "v"(bs[10]), [b11] "v"(bs[11]), [b12] "v"(bs[12]), [b13] "v"(bs[13]), [b14] "v"(bs[14]), [b15] "v"(bs[15]));
}

// the DPP coefficient registers of staged candidate c (sh_dots_dpp): lane l, coefficient l % 16 per channel
template <bool SH>
__device__ inline void sh_load_dpp(const Stage* stg, uint32_t c, float cv[3]) {
#if GSRT_DPP_SH
    if (SH) {
        const uint32_t k = lane_id() & 15u;
        cv[0] = stg->sh[c][0][k];
        cv[1] = stg->sh[c][1][k];
        cv[2] = stg->sh[c][2][k];
        return;
    }
#endif
    (void)stg; (void)c;
    cv[0] = cv[1] = cv[2] = 0.0f;
}

// ---- GSRT_MFMA_SH shading
// Shade the candidates 0..m of an MFMA stage (SH, production path) for every lane's ray: as shade_stage (g
// first, wave-uniform skips), with the stage's SH sums from stage_sh_mfma. The alphas of all candidates are
// computed before the sums are read, so that the slab tests and exponentials overlap the matrix-core work.
template <bool LUT>
__device__ inline void shade_stage_m(const StageM* stg, uint32_t m, const float* lut_s, CorRay& ray, uint32_t lane) {
    float gv[kGroup];
    bool okg[kGroup];
#pragma unroll
    for (uint32_t c = 0; c < kGroup; ++c) {
        const float4 q2 = reinterpret_cast<const float4*>(&stg->rec[c])[2];  // ppx, ppy, A/2, B
        const float c2 = stg->rec[c].c, cut = LUT ? kGMax : stg->rec[c].gcut;
        const float dx = ray.pxs - q2.x, dy = ray.pys - q2.y;
        gv[c] = fmaf(c2 * dy, dy, fmaf(q2.w * dx, dy, (q2.z * dx) * dx));
        okg[c] = c < m && __float_as_uint(gv[c]) <= __float_as_uint(cut);  // see shade_stage
    }
    if (!__ballot(okg[0] || okg[1] || okg[2] || okg[3])) return;
    float sums[16];
    stage_sh_mfma(stg, ray.bs, lane, sums);
    float alpha[kGroup];
#pragma unroll
    for (uint32_t c = 0; c < kGroup; ++c) {
        alpha[c] = 0.0f;
        if (!__ballot(okg[c])) continue;
        const float4 q0 = reinterpret_cast<const float4*>(&stg->rec[c])[0];  // lo, depth
        const float4 q1 = reinterpret_cast<const float4*>(&stg->rec[c])[1];  // hi, opacity
        const float lo[3] = {q0.x, q0.y, q0.z}, hi[3] = {q1.x, q1.y, q1.z};
        const bool ok = okg[c] & slab_hit_rel(ray.R, lo, hi);
        const float gs = ok ? gv[c] : 0.0f;
        const float e = LUT ? linear_exp(lut_s, gs) : exp_neg_nocheck(-gs);
        float a = q1.w * e;
        if (a > 0.99f) a = 0.99f;
        alpha[c] = (ok && a > kAlphaMin) ? a : 0.0f;
    }
#pragma unroll
    for (uint32_t c = 0; c < kGroup; ++c) {
        // front to back: a ray that stopped at an earlier candidate (active false) takes no more hits
        const bool contrib = alpha[c] > 0.0f && ray.active;
        const float tn = ray.T * (1.0f - alpha[c]);
        const bool term = contrib && tn < 1e-4f;
        if (contrib && !term) {
            float col[3];
#pragma unroll
            for (uint32_t ch = 0; ch < 3; ++ch) {
                const float v = sums[3 * c + ch] + 0.5f;
                col[ch] = v > 0.0f ? v : 0.0f;
            }
            const float w = alpha[c] * ray.T;
            ray.C[0] = fmaf(col[0], w, ray.C[0]);
            ray.C[1] = fmaf(col[1], w, ray.C[1]);
            ray.C[2] = fmaf(col[2], w, ray.C[2]);
            ray.T = tn;
        }
        if (term) {
            ray.active = false;
            ray.pxs = __builtin_nanf("");
        }
    }
}

// the slab-free flags (bit 31 of a tile-list entry) of the stage starting at g0, as a wave-uniform bit mask
__device__ inline uint32_t stage_flags(const uint32_t* ids, uint32_t count, uint32_t g0, uint32_t lane) {
    const bool f = lane < kGroup && g0 + lane < count && (ids[g0 + lane] >> 31) != 0u;
    return (uint32_t)__ballot(f);
}
#ifdef GSRT_X_SLABFREE
#define GSRT_STAGE_FLAGS(g) stage_flags(ids, count, (g), lane)
#else
#define GSRT_STAGE_FLAGS(g) 0u
#endif

// ---- GSRT_X_SLABFREE
// Tiles of a group every one of whose rays meets the splat's AABB, so that their per-ray slab test can be skipped
// (the result is the same: it would pass for every ray). The rays through a pixel rectangle form the convex cone
// spanned by its four corner rays, and the rays meeting a convex box form a convex cone too: if the four corner
// rays meet the box shrunk by a margin, every ray of the tile meets the shrunk box exactly, and the f32 slab test
// of ray_box_test (vulkan_ray_tracing.cc:217-237) on the real box then passes, its rounding (a few ulps of
// |lo|, |hi| per axis) lying far inside the margin (1e-3 of the extent + 1e-5 of the coordinates). The ray
// segment bounds [tmin, tmax] are left out of the cone argument by requiring the whole box to lie between 2 tmin
// and tmax / 2 from the origin. Bit t of the result: tile t (row-major in the group) is slab-free.
__device__ inline uint32_t slab_free_tiles(const SplatRec* rec, const ObjRay* cray) {
    const float4* r4 = reinterpret_cast<const float4*>(rec);
    const float4 q0 = r4[0], q1 = r4[1];
    const float lo[3] = {q0.x, q0.y, q0.z}, hi[3] = {q1.x, q1.y, q1.z};  // relative to the camera origin
    float slo[3], shi[3], near2 = 0.0f, far2 = 0.0f;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float mag = fmaxf(fabsf(lo[k]), fabsf(hi[k]));
        const float dl = fmaf(1e-3f, hi[k] - lo[k], 1e-5f * mag);
        slo[k] = lo[k] + dl;
        shi[k] = hi[k] - dl;
        ok = ok && slo[k] < shi[k];
        const float nk = lo[k] > 0.0f ? lo[k] : (hi[k] < 0.0f ? -hi[k] : 0.0f);
        near2 = fmaf(nk, nk, near2);
        far2 = fmaf(mag, mag, far2);
    }
    const float tmn = 2.0f * cray[0].tmin, tmx = 0.5f * cray[0].tmax;
    ok = ok && near2 > tmn * tmn && far2 < tmx * tmx;
    if (!__ballot(ok)) return 0u;
    uint32_t corners = 0;
    if (ok) {
#pragma unroll 5
        for (uint32_t c = 0; c < (kFG + 1) * (kFG + 1); ++c)
            corners |= slab_hit_rel(cray[c], slo, shi) ? (1u << c) : 0u;
    }
    uint32_t sf = 0;
#pragma unroll
    for (uint32_t t = 0; t < kFG * kFG; ++t) {
        const uint32_t c = (t / kFG) * (kFG + 1) + t % kFG;  // top-left corner of tile t
        const uint32_t need = (1u << c) | (1u << (c + 1)) | (1u << (c + kFG + 1)) | (1u << (c + kFG + 2));
        sf |= (corners & need) == need ? (1u << t) : 0u;
    }
    return sf;
}

// ---- GSRT_REC_SMEM (round 3): the shading loop's records as scalar loads
// A candidate is wave-uniform, so its 64-B SplatRec can be read through the constant address space (s_load into
// SGPRs, taken by the VALU as operands) instead of LDS-DMA + 16-B broadcast reads; the stage then carries only the
// SH rows (one DMA of 48 pieces). Bit-exact (the GPU parity tests passed with it), but slower. C3, same box:
// render kernel 1.344 -> 1.437 ms (frame 6006 -> 5630 Mrays/s), C2 -3 %. PMC per C3 wave (profiles/README.md):
// SQ_LDS_IDX_ACTIVE 4722 -> 3362 (-29 %), LDS instructions 1083 -> 850, but SMEM 41 -> 266, SALU 1948 -> 2377
// (+22 %: scalar address math and SGPR spills) and SQ_WAIT_ANY 12144 -> 15654 cycles (+29 %). LDS reads and scalar
// loads share lgkmcnt, and scalar loads return out of order, so every wait is lgkmcnt(0): a stage's records can
// be neither prefetched past the SH reads nor overlapped with them, and their latency is exposed per stage.
// Last commit with it in place: 175935d (gsrt_render.hip, -DGSRT_REC_SMEM=1).
// #if GSRT_REC_SMEM
// typedef const __attribute__((address_space(4))) SplatRec* ConstRecs;  // constant address space: scalar loads
// 
// // shade_stage with the records read as scalar loads (GSRT_REC_SMEM): the same operations in the same order on
// // the same values, so the results are bit-identical; only the operands' home differs (SGPRs instead of LDS).
// // sids: the stage's kGroup ids in LDS (16-B aligned). Ids past m are replaced by the first (never used: their
// // g test fails on c >= m), so no load leaves the record array.
// template <bool SH, bool LUT>
// __device__ inline void shade_stage_smem(const Stage* stg, const uint32_t* sids, uint32_t m, const float* lut_s,
//                                         CorRay& ray, const SplatRec* recs) {
//     const ConstRecs R = (ConstRecs)recs;
//     const uint4 iv = *reinterpret_cast<const uint4*>(sids);
//     uint32_t id[4] = {(uint32_t)__builtin_amdgcn_readfirstlane(iv.x), (uint32_t)__builtin_amdgcn_readfirstlane(iv.y),
//                       (uint32_t)__builtin_amdgcn_readfirstlane(iv.z), (uint32_t)__builtin_amdgcn_readfirstlane(iv.w)};
//     static_assert(kGroup == 4, "four ids per stage");
// #pragma unroll
//     for (uint32_t c = 1; c < kGroup; ++c) id[c] = c < m ? id[c] : id[0];
//     float gv[kGroup];
//     bool okg[kGroup];
// #pragma unroll
//     for (uint32_t c = 0; c < kGroup; ++c) {
//         const float ppx = R[id[c]].ppx, ppy = R[id[c]].ppy, a2 = R[id[c]].a, b = R[id[c]].b;
//         const float c2 = R[id[c]].c, cut = LUT ? kGMax : R[id[c]].gcut;
//         const float dx = ray.pxs - ppx, dy = ray.pys - ppy;
//         gv[c] = fmaf(c2 * dy, dy, fmaf(b * dx, dy, (a2 * dx) * dx));
//         okg[c] = c < m && __float_as_uint(gv[c]) <= __float_as_uint(cut);
//     }
// #pragma unroll
//     for (uint32_t c = 0; c < kGroup; ++c) {
//         if (!__ballot(okg[c])) continue;
//         const float lo[3] = {R[id[c]].lo[0], R[id[c]].lo[1], R[id[c]].lo[2]};
//         const float hi[3] = {R[id[c]].hi[0], R[id[c]].hi[1], R[id[c]].hi[2]};
//         const float op = R[id[c]].opacity;
//         const bool ordered = (int)__float_as_uint(op) >= 0;  // wave-uniform already (a scalar load)
//         const bool ok = okg[c] & (ordered ? slab_hit_ordered(ray.R, lo, hi) : slab_hit_rel(ray.R, lo, hi));
//         const float gs = LUT ? (ok ? gv[c] : 0.0f) : gv[c];
//         const float e = LUT ? linear_exp(lut_s, gs) : exp_neg_nocheck(-gs);
//         const float a = __builtin_fminf(fabsf(op) * e, 0.99f);
//         const bool contrib = ok && a > kAlphaMin;
//         const float alpha = contrib ? a : 0.0f;
//         if (blend_hit<SH, false>(stg, c, alpha, contrib, ray)) {
// #pragma unroll
//             for (uint32_t c1 = c + 1; c1 < kGroup; ++c1) okg[c1] = false;
//         }
//     }
// }
// #endif
// 
// template <bool SH, bool NOREC = false>
// __device__ inline void stage_issue(const uint32_t* ids, uint32_t count, uint32_t g0, uint32_t lane, Stage* dst,
//                                    const SplatRec* recs, const float* sh) {
//     if (NOREC) {  // SH rows only (GSRT_REC_SMEM): piece p is row piece p % 12 of candidate g0 + p / 12, at 16 p
//         static_assert(12 * kGroup <= 64, "one DMA instruction per stage");
//         if (!SH) return;
//         const uint32_t p = lane < 12 * kGroup ? lane : 0u;  // lane 0 always loads
//         uint32_t c = g0 + p / 12;
//         c = c < count ? c : g0;
//         if (lane < 12 * kGroup || lane == 0)
//             __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const char*>(sh) + (size_t)ids[c] * 192u +
//                                                            (p % 12) * 16u),
//                                              (void*)(reinterpret_cast<char*>(dst->sh)), 16, 0, 0);
//         return;
//     }
