// gsrt_project.hpp -- the per-splat COR/REF projection (device code), shared by k_project (gsrt_scene.hip) and the
// fused prep kernel k_prep_cor (gsrt_render.hip: frontier blocks + projection blocks in one launch).
#pragma once

#include "gsrt_internal.hpp"

namespace gsrt {

// REF projection: the per-Gaussian half of RayTracing.ProceduralGauss.rint:62-102, exactly as written
// there (fx and fy both scale by Height; V is the 2D covariance itself, not its inverse).
__device__ GSRT_INLINE void project_ref(const gsrt_ubo& u, const gsrt_gauss_param& g, SplatRec& s) {
    const float* MV = u.model_view;
    const float* P = u.projection;
    const float c4[4] = {g.center_opacity[0], g.center_opacity[1], g.center_opacity[2], 1.0f};
    float t[4];
    mul4v(MV, c4, t);
    s.depth = t[2];
    s.opacity = g.center_opacity[3];
    float ph[4];
    mul4v(P, t, ph);
    const float ndcx = ph[0] / ph[3], ndcy = ph[1] / ph[3];
    s.ppx = ((ndcx + 1.0f) * (float)u.width) * 0.5f;
    s.ppy = ((ndcy + 1.0f) * (float)u.height) * 0.5f;
    const float fx = (cm(P, 0, 0) * (float)u.height) * 0.5f;
    const float fy = (cm(P, 1, 1) * (float)u.height) * 0.5f;
    const float zz = t[2] * t[2];
    const float J[9] = {fx / t[2], 0.0f, 0.0f, 0.0f, fy / t[2], 0.0f, (-fx * t[0]) / zz, (-fy * t[1]) / zz, 0.0f};
    float W[9];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) W[c * 3 + r] = cm(MV, c, r);
    const float* cv = g.cov3d;
    const float Sg[9] = {cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]};
    float T[9], TS[9], V[9];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            T[c * 3 + r] = (J[0 * 3 + r] * W[c * 3 + 0] + J[1 * 3 + r] * W[c * 3 + 1]) + J[2 * 3 + r] * W[c * 3 + 2];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            TS[c * 3 + r] = (T[0 * 3 + r] * Sg[c * 3 + 0] + T[1 * 3 + r] * Sg[c * 3 + 1]) + T[2 * 3 + r] * Sg[c * 3 + 2];
    // V = TS * transpose(T): V[c][r] = (TS[0][r]*T[0][c] + TS[1][r]*T[1][c]) + TS[2][r]*T[2][c]
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            V[c * 3 + r] = (TS[0 * 3 + r] * T[0 * 3 + c] + TS[1 * 3 + r] * T[1 * 3 + c]) + TS[2 * 3 + r] * T[2 * 3 + c];
    s.a = V[0];  // V[0][0]
    s.b = V[1];  // V[0][1]
    s.c = V[4];  // V[1][1]
    s.valid = 1u;
}

// COR projection: depth = -view z, Jacobian of the actual pixel mapping (fx = P00 W/2, fy = P11 H/2),
// V += 0.3 I low-pass, conic = V^-1 (COR flags).
__device__ GSRT_INLINE void project_cor(const gsrt_ubo& u, const gsrt_gauss_param& g, SplatRec& s) {
    const float* MV = u.model_view;
    const float* P = u.projection;
    const float c4[4] = {g.center_opacity[0], g.center_opacity[1], g.center_opacity[2], 1.0f};
    float t[4];
    mul4v(MV, c4, t);
    s.valid = 0u;
    s.depth = -t[2];
    s.opacity = g.center_opacity[3];
    s.ppx = s.ppy = s.a = s.b = s.c = 0.0f;
    if (!(s.depth > 0.0f)) return;
    float ph[4];
    mul4v(P, t, ph);
    const float ndcx = ph[0] / ph[3], ndcy = ph[1] / ph[3];
    s.ppx = ((ndcx + 1.0f) * (float)u.width) * 0.5f;
    s.ppy = ((ndcy + 1.0f) * (float)u.height) * 0.5f;
    const float fx = (cm(P, 0, 0) * (float)u.width) * 0.5f;
    const float fy = (cm(P, 1, 1) * (float)u.height) * 0.5f;
    const float id = 1.0f / s.depth;
    const float id2 = id * id;
    const float j00 = fx * id, j02 = (fx * t[0]) * id2, j11 = fy * id, j12 = (fy * t[1]) * id2;
    float T0[3], T1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        T0[k] = fmaf(j02, cm(MV, k, 2), j00 * cm(MV, k, 0));
        T1[k] = fmaf(j12, cm(MV, k, 2), j11 * cm(MV, k, 1));
    }
    const float* cv = g.cov3d;
    const float Sg[9] = {cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]};
    float u0[3], u1[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        u0[r] = fmaf(Sg[r * 3 + 2], T0[2], fmaf(Sg[r * 3 + 1], T0[1], Sg[r * 3 + 0] * T0[0]));
        u1[r] = fmaf(Sg[r * 3 + 2], T1[2], fmaf(Sg[r * 3 + 1], T1[1], Sg[r * 3 + 0] * T1[0]));
    }
    const float v00 = fmaf(T0[2], u0[2], fmaf(T0[1], u0[1], T0[0] * u0[0])) + 0.3f;
    const float v01 = fmaf(T0[2], u1[2], fmaf(T0[1], u1[1], T0[0] * u1[0]));
    const float v11 = fmaf(T1[2], u1[2], fmaf(T1[1], u1[1], T1[0] * u1[0])) + 0.3f;
    const float det = fmaf(v00, v11, -(v01 * v01));
    if (!(det > 0.0f)) return;
    const float idet = 1.0f / det;
    s.a = v11 * idet;
    s.b = -v01 * idet;
    s.c = v00 * idet;
    s.valid = 1u;
}

// One wave per workgroup and <= 80 VGPRs (6 waves/SIMD): the COR projection of frame f+1 runs on the prep
// stream beside frame f's render kernel (80 VGPRs, one-wave workgroups), so each of its workgroups must fit
// into the slot one retiring render wave frees; a 4-wave workgroup would wait for the render kernel's tail.
// wave issue priority of the prep kernels (k_prep_cor, k_frontier, k_group_list, k_project, k_copy_rows): above the
// render kernel's, so their latency chains advance while they share SIMDs with render waves
constexpr int kPrepSetprio = 3;
// Cheap early test of a rank of a sharded frame (k_project): may a tile of this rank see the splat? A pixel box
// that contains the projection of the AABB, from the AABB in view space (centre + |rotation| extents) and the
// extreme ratios X / depth, Y / depth over it, widened by 1e-3 relative + 2 px for rounding. The exact footprint
// (project_one below) lies inside the projection of the AABB whenever the box is in front of the camera, so a
// splat this test rejects is one the exact test rejects too. Boxes reaching the camera plane, and projections
// other than the plain perspective form (P00, P11 and w = -z), always go on to the exact test.
__device__ GSRT_INLINE bool may_own_box(const gsrt_ubo& u, const gsrt_aabb& a, const RankTiles& own) {
    const float* MV = u.model_view;
    const float* P = u.projection;
    const bool plain = cm(P, 1, 0) == 0.0f && cm(P, 2, 0) == 0.0f && cm(P, 3, 0) == 0.0f && cm(P, 0, 1) == 0.0f &&
                       cm(P, 2, 1) == 0.0f && cm(P, 3, 1) == 0.0f && cm(P, 0, 3) == 0.0f && cm(P, 1, 3) == 0.0f &&
                       cm(P, 2, 3) == -1.0f && cm(P, 3, 3) == 0.0f;
    if (!plain) return true;
    const float c[3] = {0.5f * (a.min_x + a.max_x), 0.5f * (a.min_y + a.max_y), 0.5f * (a.min_z + a.max_z)};
    const float e[3] = {0.5f * (a.max_x - a.min_x), 0.5f * (a.max_y - a.min_y), 0.5f * (a.max_z - a.min_z)};
    float vc[3], ve[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        vc[r] = cm(MV, 0, r) * c[0] + cm(MV, 1, r) * c[1] + cm(MV, 2, r) * c[2] + cm(MV, 3, r);
        ve[r] = (fabsf(cm(MV, 0, r)) * e[0] + fabsf(cm(MV, 1, r)) * e[1] + fabsf(cm(MV, 2, r)) * e[2]) * 1.001f +
                1e-6f * (fabsf(vc[r]) + 1.0f);
    }
    const float d0 = -vc[2] - ve[2], d1 = -vc[2] + ve[2];  // depth range
    if (!(d0 > 1e-3f * (fabsf(d1) + 1.0f))) return true;    // reaches the camera plane (or NaN): the exact test
    const float id0 = 1.0f / d0, id1 = 1.0f / d1;
    auto range = [&](float lo, float hi, float& r0, float& r1) {  // extreme lo..hi / depth over [d0, d1]
        r0 = lo >= 0.0f ? lo * id1 : lo * id0;
        r1 = hi >= 0.0f ? hi * id0 : hi * id1;
    };
    float rx0, rx1, ry0, ry1;
    range(vc[0] - ve[0], vc[0] + ve[0], rx0, rx1);
    range(vc[1] - ve[1], vc[1] + ve[1], ry0, ry1);
    const float W = (float)u.width, H = (float)u.height, p00 = cm(P, 0, 0), p11 = cm(P, 1, 1);
    float x0 = (p00 * rx0 + 1.0f) * 0.5f * W, x1 = (p00 * rx1 + 1.0f) * 0.5f * W;
    float y0 = (p11 * ry0 + 1.0f) * 0.5f * H, y1 = (p11 * ry1 + 1.0f) * 0.5f * H;
    if (x0 > x1) { const float t = x0; x0 = x1; x1 = t; }
    if (y0 > y1) { const float t = y0; y0 = y1; y1 = t; }
    const float mx = 1e-3f * fmaxf(fabsf(x0), fabsf(x1)) + 2.0f, my = 1e-3f * fmaxf(fabsf(y0), fabsf(y1)) + 2.0f;
    return rank_owns_box(x0 - mx, x1 + mx, y0 - my, y1 + my, own);
}

// the sort key of leaf i in its parent node (k_group_list's traversal reads it there)
__device__ GSRT_INLINE void put_node_key(BvhNode* nodes, const uint32_t* gid_slot, uint32_t i, uint32_t depth_bits) {
    const uint32_t slot = gid_slot[i];
    reinterpret_cast<uint32_t*>(nodes + (slot & ~kLeafBit))[(slot >> 31) ? 15 : 11] = depth_bits;
}
// the sort key and the footprint box of leaf i in its parent node: the box {x0, x1, y0, y1} takes the leaf's box
// slot (words lo[0], lo[1], lo[2], hi[0]), so a COR traversal tests the footprint where it would test the AABB
// (leaf_fp_meets) and needs no footprint load; the slot's fit writes the AABB back (gsrt_scene::slot_leaf_fp)
__device__ GSRT_INLINE void put_node_key_fp(BvhNode* nodes, const uint32_t* gid_slot, uint32_t i, uint32_t depth_bits,
                                       float4 fp) {
    const uint32_t slot = gid_slot[i];
    const bool right = (slot >> 31) != 0;
    float* node = reinterpret_cast<float*>(nodes + (slot & ~kLeafBit));
    float* w = node + (right ? 8 : 0);  // the leaf's box slot: lo at words 0-2, hi at 4-6 of w
    w[0] = fp.x; w[1] = fp.y; w[2] = fp.z; w[4] = fp.w;
    reinterpret_cast<uint32_t*>(node)[right ? 15 : 11] = depth_bits;  // l_key / r_key
}

// Projection of splat i. Returns whether the splat may hold a finite key in this slot (the keyed bitmap, see
// k_project); prev = its bit from the slot's previous projection (true when unknown).
template <int MODE>
__device__ GSRT_INLINE bool project_one(uint32_t i, uint32_t n, const gsrt_ubo& ubo, const gsrt_gauss_param* __restrict__ params,
                                   const gsrt_aabb* __restrict__ aabbs, SplatRec* __restrict__ recs,
                                   BvhNode* __restrict__ nodes, const uint32_t* __restrict__ gid_slot,
                                   float4* __restrict__ footprint, const RankTiles& own, bool prev,
                                   bool leaf_fp = false, uint32_t* __restrict__ depth_unsafe = nullptr) {
    const gsrt_aabb a = aabbs[i];
    if (MODE != GSRT_MODE_REF && footprint && own.active && !may_own_box(ubo, a, own)) {
        // a rank of a sharded frame: no tile of this rank can see the splat. Like a projected splat that is not the
        // rank's (below), its keys become +inf, which the traversals reject -- written only when they may not be
        // +inf already (prev): in steady state a splat outside the rank's super-tiles costs one 24-B read
        if (prev) {
            if (nodes) put_node_key(nodes, gid_slot, i, 0x7f800000u);
            recs[i].depth = __uint_as_float(0x7f800000u);
        }
        return false;
    }
    const gsrt_gauss_param g = params[i];
    SplatRec s;
    if (MODE == GSRT_MODE_REF) {
        project_ref(ubo, g, s);
    } else {
        project_cor(ubo, g, s);
        if (!s.valid) s.depth = __int_as_float(0x7f800000);  // +inf: the traversal key test rejects it
        bool mine = true;  // some tile this rank renders can see the splat (multi-GPU: RankTiles)
        if (footprint) {
            // Conservative pixel box of where the splat can contribute, the intersection of
            //  (1) the g-ellipse: alpha > 1/255 needs g <= G = min(5.6, ln(255 op)); {g <= G} is d^T Q d <= 2G
            //      (Q = conic), half-extents sqrt(2G Q^-1_xx), sqrt(2G Q^-1_yy), widened by 1 % + 0.01 px;
            //  (2) the projected AABB: a ray through pixel coordinate (x, y) meets the box only if (x, y) lies
            //      in the box's projection, bounded by its 8 projected corners when all lie in front of the
            //      camera (the ray convention of GaussTracing.rgen:39-43: x = (ndc + 1) W / 2), widened by
            //      1e-3 relative + 0.01 px.
            //  (3) the ellipse itself for the exact ellipse-rectangle test of k_render's fp_meets / ell_meets:
            //      (ppx, ppy, B/C, B/A), (C/T, A/T, det/(C T), det/(A T)).
            float4 fp = make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);  // empty: never meets a tile
            float4 eu = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ev = eu;
            const float op255 = s.opacity * 255.0f;
            if (s.valid && op255 > 1.0f) {
                const float G = fminf(kGMax, logf(op255) + 0.01f);
                const float det = s.a * s.c - s.b * s.b;
                if (det > 0.0f) {
                    const float q = 2.0f * G / det;
                    const float hx = sqrtf(q * s.c) * 1.01f + 0.01f, hy = sqrtf(q * s.a) * 1.01f + 0.01f;
                    fp = make_float4(s.ppx - hx, s.ppx + hx, s.ppy - hy, s.ppy + hy);
                    // the ellipse for k_render's ell_meets: 2g = d^T Q d <= 2G, threshold widened to
                    // T = 2G * 1.02 + 2e-3 (covers the f32 rounding of the per-ray g at condition numbers < 1e4);
                    // the edge-restricted forms use det / C and det / A (computed in f64: det = AC - B^2 cancels)
                    float bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
                    bool front = true;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const float w4[4] = {k & 1 ? a.max_x : a.min_x, k & 2 ? a.max_y : a.min_y, k & 4 ? a.max_z : a.min_z, 1.0f};
                        float v[4], h[4];
                        mul4v(ubo.model_view, w4, v);
                        mul4v(ubo.projection, v, h);
                        front = front && h[3] > 1e-6f && -v[2] > 1e-6f;
                        const float x = (h[0] / h[3] + 1.0f) * (float)ubo.width * 0.5f;
                        const float y = (h[1] / h[3] + 1.0f) * (float)ubo.height * 0.5f;
                        bx0 = fminf(bx0, x); bx1 = fmaxf(bx1, x); by0 = fminf(by0, y); by1 = fmaxf(by1, y);
                    }
                    if (front) {
                        const float mx = 1e-3f * fmaxf(fabsf(bx0), fabsf(bx1)) + 0.01f;
                        const float my = 1e-3f * fmaxf(fabsf(by0), fabsf(by1)) + 0.01f;
                        fp.x = fmaxf(fp.x, bx0 - mx); fp.y = fminf(fp.y, bx1 + mx);
                        fp.z = fmaxf(fp.z, by0 - my); fp.w = fminf(fp.w, by1 + my);
                    }
                    // (after the corner loop: the f64 temporaries and eu / ev are not live across it)
                    const double A = s.a, B = s.b, C = s.c, dd = A * C - B * B;
                    const double T = 2.0 * (double)G * 1.02 + 2e-3;
                    eu = make_float4(s.ppx, s.ppy, (float)(B / C), (float)(B / A));
                    ev = make_float4((float)(C / T), (float)(A / T), (float)(dd / (C * T)), (float)(dd / (A * T)));
                    if (A * C > 1e4 * dd) ev = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // ill-conditioned: box only
                }
            }
            // a rank of a sharded frame projects every splat but keeps only those whose footprint box meets a
            // super-tile with a tile of its own (the others get depth +inf: their keys reject them in the traversal,
            // the record's other words and the footprint are not written, ~7/8 of the writes at 8 ranks)
            mine = rank_owns_box(fp.x, fp.y, fp.z, fp.w, own);
            if (mine) {
                float4* rec = footprint + kFpWords * (size_t)i;  // one 64-B record per splat
                rec[0] = fp;
                rec[1] = eu;
                rec[2] = ev;
                // leaf_fp: the key with this frame's box (a finite key always comes with it; an +inf key's box is
                // never read, the traversal's key test rejects it first)
                if (nodes && leaf_fp) put_node_key_fp(nodes, gid_slot, i, __float_as_uint(s.depth), fp);
            }
        }
        if (!mine) s.depth = __int_as_float(0x7f800000);
        // the traversals' depth cull bounds a subtree's keys by its box (depth_lo): sound while every keyed centre lies
        // within its own AABB's bound, which only a caller-supplied AABB that misses its centre breaks
        if (depth_unsafe && s.depth < depth_lo(zrow_of(ubo.model_view), &a.min_x, &a.max_x)) atomicOr(depth_unsafe, 1u);
        if (nodes && (mine || prev) && !(mine && leaf_fp && footprint))
            put_node_key(nodes, gid_slot, i, __float_as_uint(s.depth));  // next to its box
        if (!mine) {
            if (prev) recs[i].depth = s.depth;  // the render kernel's own traversal keys (KeyCorRec) read it
            return false;
        }
        s.a *= 0.5f;  // pre-scaled conic (SplatRec): exact
        s.c *= 0.5f;
    }
    float o[3];
    ray_origin(ubo, o);
    s.lo[0] = a.min_x - o[0]; s.lo[1] = a.min_y - o[1]; s.lo[2] = a.min_z - o[2];
    s.hi[0] = a.max_x - o[0]; s.hi[1] = a.max_y - o[1]; s.hi[2] = a.max_z - o[2];
    s.gcut = 0.0f; s.pad1 = 0u;
    // clamped at +0 so that k_render_cor tests g in [0, gcut] as one unsigned compare (an opacity below 1/255
    // then passes only g = +0, and its alpha = opacity <= 1/255 is dropped by the alpha test as before)
    if (MODE != GSRT_MODE_REF && s.valid) s.gcut = fmaxf(0.0f, fminf(kGMax, logf(s.opacity * 255.0f) + 0.01f));
    if (MODE != GSRT_MODE_REF) {
        // a box strictly on one side of the origin on every axis is stored as (near, far) per axis for the rays
        // that can reach it (k_render_cor's slab_hit_ordered); one that touches or straddles an axis plane through
        // the origin keeps (lo, hi) and is flagged by a negated opacity word (the general slab test, which is
        // symmetric in lo and hi, serves both layouts; every reader of a COR opacity takes |opacity|)
        bool ordered = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (s.hi[k] < 0.0f) {
                const float t = s.lo[k];
                s.lo[k] = s.hi[k];
                s.hi[k] = t;
            } else if (!(s.lo[k] > 0.0f)) {
                ordered = false;
            }
        }
        if (!ordered) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {  // back to (lo, hi) on every axis
                if (s.lo[k] > s.hi[k]) {
                    const float t = s.lo[k];
                    s.lo[k] = s.hi[k];
                    s.hi[k] = t;
                }
            }
            s.opacity = -s.opacity;
        }
    }
    recs[i] = s;
    return true;
}

}  // namespace gsrt
