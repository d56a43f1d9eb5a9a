"""An independent float64 restatement of the COR render ("COR flags") -- test infrastructure.

It shares no code and no operation order with oracle/gsrt_oracle.c or the HIP kernels: every quantity is computed
in float64 with numpy's own formulas, the exponential is np.exp, candidates are found by brute force over all
Gaussians, and the blend walks each ray's hits in (depth, id) order. The structure it follows is the reference's:
  - Gaussian covariance and AABB: Gauss::init_cov3d / init_radius (RayTracingInVulkan/src/Assets/Sphere.hpp:129-165);
  - primary rays with the pixel jitter of RayTracing.rgen:27-43 (RandomFloat / RandomInt, Random.glsl:24-37;
    every pixel starts from Camera.RandomSeed);
  - candidate set: the exact AABB slab test on [0.001, 10000] (vulkan_ray_tracing.cc:217-237);
  - per candidate, the EWA projection of RayTracing.ProceduralGauss.rint:62-102 with the COR flags: depth = -view z,
    the true Jacobian (fx = P00 W/2, fy = P11 H/2), V + 0.3 I, conic = (V + 0.3 I)^-1, g = 1/2 d^T conic d,
    0 <= g <= 5.6, alpha = min(opacity exp(-g), 0.99), kept when alpha > 1/255;
  - front-to-back blend (rchit:15-33 with the COR flags): C += T alpha colour, T *= 1 - alpha, stop before a hit
    that would take T below 1e-4; colour = max(0, 0.5 + sum_k sh_k Y_k(dir)) (3DGS SH-3 basis) or 1 without SH;
    output (C, 1 - T) averaged over the samples.

Decisions that float32 rounding can flip are reported per pixel and those pixels are excluded from the comparison
(SURVEY.md §8c): an alpha within `alpha_rel` of 1/255, a T(1 - alpha) within `trans_rel` of 1e-4, a slab test
within `slab_rel` of its boundary, two contributing hits of different colour whose depths differ by less than
`depth_rel` (their float32 order can swap), and a projection whose determinant is within `det_rel` of zero.
"""
import numpy as np

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def covariance(rot, scale):
    """Sigma = (S R)^T (S R) with R the glm::mat3 Sphere.hpp:143-147 builds from (r, x, y, z), in float64."""
    q = np.asarray(rot, np.float64)
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    # glm's mat3 constructor is column-major: argument k lands in column k // 3, row k % 3
    cols = np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        np.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        np.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -1)  # [n, row, col]
    M = np.asarray(scale, np.float64)[:, :, None] * cols  # S * R: row i of R scaled by s_i
    return np.einsum("nki,nkj->nij", M, M)


def _mat(a):
    return np.asarray(a, np.float64).reshape(4, 4).T  # column-major storage -> math matrix


class Ubo:
    def __init__(self, ubo):
        u = ubo.reshape(-1)[0] if ubo.dtype.names else ubo
        self.MV = _mat(u["model_view"])
        self.P = _mat(u["projection"])
        self.MVi = _mat(u["model_view_inverse"])
        self.Pi = _mat(u["projection_inverse"])
        self.W, self.H = int(u["width"]), int(u["height"])
        self.S = max(1, int(u["samples"]))
        self.seed = int(u["random_seed"])
        self.focus = float(u["focus_distance"])


def jitter(seed, samples):
    """RandomFloat pairs from the LCG, x first then y (RayTracing.rgen:38)."""
    out = []
    s = seed & 0xFFFFFFFF
    for _ in range(samples):
        pair = []
        for _ in range(2):
            s = (1664525 * s + 1013904223) & 0xFFFFFFFF
            pair.append((s & 0xFFFFFF) / float(1 << 24))
        out.append(pair)
    return out


def rays(u, px, py):
    """origin (3,) and unit directions (n, 3) for pixel coordinates px, py (float64 arrays)."""
    uv = np.stack([px / u.W * 2.0 - 1.0, py / u.H * 2.0 - 1.0, np.ones_like(px), np.ones_like(px)], -1)
    tg = uv @ u.Pi.T
    v = tg[:, :3] * u.focus
    v = v / np.linalg.norm(v, axis=1, keepdims=True)
    d = v @ u.MVi[:3, :3].T
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    o = u.MVi[:3, 3]
    return o, d


def sh_basis(d):
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    xx, yy, zz = x * x, y * y, z * z
    return np.stack([
        np.full_like(x, SH_C0), -SH_C1 * y, SH_C1 * z, -SH_C1 * x,
        SH_C2[0] * x * y, SH_C2[1] * y * z, SH_C2[2] * (2 * zz - xx - yy), SH_C2[3] * x * z, SH_C2[4] * (xx - yy),
        SH_C3[0] * y * (3 * xx - yy), SH_C3[1] * x * y * z, SH_C3[2] * y * (4 * zz - xx - yy),
        SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy), SH_C3[4] * x * (4 * zz - xx - yy), SH_C3[5] * z * (xx - yy),
        SH_C3[6] * x * (xx - 3 * yy)], -1)


class Splats:
    """Per-Gaussian screen-space quantities (the rint projection with the COR flags), float64."""

    def __init__(self, u, center, rot, scale, opacity, sh=None, det_rel=1e-6):
        c = np.asarray(center, np.float64)
        n = len(c)
        self.n = n
        rad = 3.0 * np.asarray(scale, np.float64).max(1)
        self.lo, self.hi = c - rad[:, None], c + rad[:, None]
        t = np.concatenate([c, np.ones((n, 1))], 1) @ u.MV.T
        self.depth = -t[:, 2]
        ph = t @ u.P.T
        self.ppx = (ph[:, 0] / ph[:, 3] + 1.0) * u.W / 2.0
        self.ppy = (ph[:, 1] / ph[:, 3] + 1.0) * u.H / 2.0
        fx, fy = u.P[0, 0] * u.W / 2.0, u.P[1, 1] * u.H / 2.0
        dd = np.where(self.depth > 0, self.depth, 1.0)
        J = np.zeros((n, 2, 3))
        J[:, 0, 0] = fx / dd
        J[:, 0, 2] = fx * t[:, 0] / dd ** 2
        J[:, 1, 1] = fy / dd
        J[:, 1, 2] = fy * t[:, 1] / dd ** 2
        T = J @ u.MV[:3, :3]
        V = T @ covariance(rot, scale) @ np.transpose(T, (0, 2, 1)) + 0.3 * np.eye(2)
        det = V[:, 0, 0] * V[:, 1, 1] - V[:, 0, 1] * V[:, 1, 0]
        self.valid = (self.depth > 0) & (det > 0)
        self.det_near = np.abs(det) <= det_rel * np.abs(V[:, 0, 0] * V[:, 1, 1])
        sd = np.where(self.valid, det, 1.0)
        self.ca, self.cb, self.cc = V[:, 1, 1] / sd, -V[:, 0, 1] / sd, V[:, 0, 0] / sd
        self.opacity = np.asarray(opacity, np.float64)
        self.sh = None if sh is None else np.asarray(sh, np.float64).reshape(n, 16, 3)


class _Subset:
    """the AABBs of some Gaussians (what _tile_candidates reads)"""

    def __init__(self, sp, idx):
        self.lo, self.hi, self.n = sp.lo[idx], sp.hi[idx], len(idx)


def _tile_candidates(u, sp, x0, x1, y0, y1):
    """Gaussians whose bounding sphere (centre, sqrt(3) x radius) meets the pyramid of all rays through the pixel
    rectangle [x0, x1] x [y0, y1]: a necessary condition for any of those rays to hit the AABB (the pyramid's side
    planes contain the origin and two corner directions; directions are a projective map of the screen point)."""
    cx = np.array([x0, x1, x1, x0], np.float64)
    cy = np.array([y0, y0, y1, y1], np.float64)
    o, d = rays(u, cx, cy)
    inner = d.mean(0)
    c = (sp.lo + sp.hi) * 0.5 - o
    rad = np.linalg.norm(sp.hi - sp.lo, axis=1) * 0.5 * (1.0 + 1e-9) + 1e-9
    keep = np.ones(sp.n, bool)
    for k in range(4):
        n = np.cross(d[k], d[(k + 1) % 4])
        n /= np.linalg.norm(n)
        if n @ inner < 0:
            n = -n
        keep &= c @ n >= -rad
    return np.nonzero(keep)[0]


def render(ubo, center, rot, scale, opacity, sh=None, rows=None, tile=16, alpha_rel=1e-3, trans_rel=1e-3,
           slab_rel=1e-5, depth_rel=1e-6):
    """RGBA (H, W, 4) float64 and a bool (H, W) mask of pixels with a decision near a threshold."""
    u = Ubo(ubo)
    sp = Splats(u, center, rot, scale, opacity, sh)
    r0, r1 = rows if rows else (0, u.H)
    out = np.zeros((u.H, u.W, 4))
    near = np.zeros((u.H, u.W), bool)
    thr_a = 1.0 / 255.0
    jit = jitter(u.seed, u.S)
    # the band's pyramid first (every tile's pyramid lies inside it), then each tile's among those
    band = _tile_candidates(u, sp, 0, u.W, r0, r1)
    sub = _Subset(sp, band)
    for ty in range(r0, r1, tile):
        for tx in range(0, u.W, tile):
            ye, xe = min(ty + tile, r1), min(tx + tile, u.W)
            cand = band[_tile_candidates(u, sub, tx, xe, ty, ye)]
            ys, xs = np.mgrid[ty:ye, tx:xe]
            xs, ys = xs.reshape(-1).astype(np.float64), ys.reshape(-1).astype(np.float64)
            m = len(xs)
            acc = np.zeros((m, 4))
            tile_near = np.zeros(m, bool)
            for jx, jy in jit:
                px, py = xs + jx, ys + jy
                o, d = rays(u, px, py)
                C = np.zeros((m, 3))
                T = np.ones(m)
                if len(cand):
                    C, T = _blend(sp, cand, px, py, o, d, tile_near, thr_a, alpha_rel, trans_rel, slab_rel, depth_rel)
                acc[:, :3] += C
                acc[:, 3] += 1.0 - T
            out[ty:ye, tx:xe] = acc.reshape(ye - ty, xe - tx, 4)
            near[ty:ye, tx:xe] = tile_near.reshape(ye - ty, xe - tx)
    return out[r0:r1] / u.S, near[r0:r1]


def _blend(sp, cand, px, py, o, d, ray_near, thr_a, alpha_rel, trans_rel, slab_rel, depth_rel):
    m = len(px)
    lo, hi = sp.lo[cand], sp.hi[cand]
    # exact slab test on [0.001, 10000], every ray against every candidate box
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0 = (lo[None, :, :] - o) * inv[:, None, :]
        t1 = (hi[None, :, :] - o) * inv[:, None, :]
    tn = np.maximum(np.nanmax(np.minimum(t0, t1), axis=2), 0.001)
    tf = np.minimum(np.nanmin(np.maximum(t0, t1), axis=2), 10000.0)
    hit = tn <= tf
    amb = np.abs(tf - tn) <= slab_rel * np.maximum(1.0, np.abs(tn))
    ri, ci = np.nonzero((hit | amb) & sp.valid[cand][None, :])
    gi = cand[ci]
    dx, dy = px[ri] - sp.ppx[gi], py[ri] - sp.ppy[gi]
    g = 0.5 * (sp.ca[gi] * dx * dx + 2.0 * sp.cb[gi] * dx * dy + sp.cc[gi] * dy * dy)
    alpha = np.minimum(sp.opacity[gi] * np.exp(-g), 0.99)
    keep = (g >= 0.0) & (g <= 5.6) & (alpha > thr_a)
    # decisions float32 may take the other way: a box grazed by a contributing splat's ray, alpha at 1/255,
    # a projection whose determinant is ~0
    a_near = np.abs(alpha / thr_a - 1.0) <= alpha_rel
    pair_amb = (amb[ri, ci] & (alpha > thr_a * (1 - alpha_rel))) | a_near | sp.det_near[gi]
    np.logical_or.at(ray_near, ri[pair_amb], True)
    sel = keep & hit[ri, ci]
    ri, gi, alpha = ri[sel], gi[sel], alpha[sel]
    order = np.lexsort((gi, sp.depth[gi], ri))  # per ray, (depth, id) order
    ri, gi, alpha = ri[order], gi[order], alpha[order]
    depth = sp.depth[gi]
    if sp.sh is not None:
        col = np.maximum(0.0, 0.5 + np.einsum("pk,pkc->pc", sh_basis(d)[ri], sp.sh[gi]))
    else:
        col = np.ones((len(ri), 3))
    # two hits whose float32 depths may compare the other way: swapping them moves the pixel by at most
    # T a1 a2 |c1 - c2| (the blend of equal colours is order-independent), so only a visible swap is ambiguous
    same = (ri[1:] == ri[:-1]) & (np.abs(depth[1:] - depth[:-1]) <= depth_rel * depth[1:])
    swing = alpha[1:] * alpha[:-1] * np.abs(col[1:] - col[:-1]).max(1)
    np.logical_or.at(ray_near, ri[1:][same & (swing > 1e-4)], True)
    # front to back: the k-th hit of every ray at once
    starts = np.searchsorted(ri, np.arange(m))
    counts = np.bincount(ri, minlength=m)
    T = np.ones(m)
    C = np.zeros((m, 3))
    live = np.ones(m, bool)
    for k in range(int(counts.max()) if len(ri) else 0):
        rr = np.nonzero(live & (counts > k))[0]
        if not len(rr):
            break
        p = starts[rr] + k
        tnext = T[rr] * (1.0 - alpha[p])
        ray_near[rr[np.abs(tnext / 1e-4 - 1.0) <= trans_rel]] = True
        stop = tnext < 1e-4
        live[rr[stop]] = False
        go, pg = rr[~stop], p[~stop]
        C[go] += (T[go] * alpha[pg])[:, None] * col[pg]
        T[go] = tnext[~stop]
    return C, T
