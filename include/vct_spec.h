/*
 * vct_spec.h — normative constants of the voxel-cone-tracing (VCT) hot path.
 *
 * The reference (fysososo/voxel-based-global-illumination) never implemented the
 * GI stages: `VoxelizationProgram` is an empty subclass
 * (assets/code/program/p_voxelization.h:4-7) and `VoxelizationRenderer::Render`
 * only draws a forward-textured mesh (assets/code/renderer/r_voxelization.cpp:4-35).
 * SURVEY.md Appendix A therefore defines the semantics; this header pins every
 * free parameter of that spec as a literal so that the HIP kernels
 * (voxel-based-global-illumination_amd/csrc) and the CPU oracle (oracle/) read the
 * SAME numbers.  Nothing here is code; it is plain C89-compatible data so the
 * C oracle, the C++ host and the HIP device code can all include it.
 *
 * Units.  All cone / DDA / SAT arithmetic is carried out in level-0 VOXEL units:
 *   q = (p - aabb_min) * inv_h,  inv_h = (float)n / extent   (float divide)
 * so a voxel has edge 1, the grid spans [0, n]^3, level l texel coords are
 * q * 2^-l - 0.5 (GL texel-centre convention).
 *
 * Floating point.  Every translation unit of the path is compiled with
 * -ffp-contract=off.  The only fused multiply-adds are the explicit fmaf()
 * calls that the spec names (trilinear accumulation, level blend, composite,
 * cone-weight accumulation, the log2 polynomial); they are exact on both the
 * host (libm / x86 FMA) and the device (v_fma_f32), so oracle and kernels can
 * agree bit for bit.
 */
#ifndef VCT_SPEC_H
#define VCT_SPEC_H

/* ---- A.6 cone marching ---------------------------------------------------- */
#define VCT_ALPHA_STOP      0.95f        /* stop when a >= 0.95                    */
#define VCT_STEP_SCALE      0.5f         /* t += 0.5 * D                            */
#define VCT_SQRT3           1.7320508f   /* t_max = n * sqrt(3) (voxel units)       */
#define VCT_SPEC_TAU_MIN    0.02f        /* specular tau = clamp(roughness, .02, 1) */
#define VCT_SPEC_TAU_MAX    1.0f

/* ---- log2 used for the mip level m = log2(D) (D >= 1) ----------------------
 * m = e + 2*s*P(s^2)/ln2 with x = 2^e * f, f in [1/sqrt2, sqrt2], s=(f-1)/(f+1)
 * P(z) = 1 + z/3 + z^2/5 + z^3/7 + z^4/9 (Horner, fmaf).  |err| < 2e-7.      */
#define VCT_LOG2_SQRT2      1.41421354f
#define VCT_INV_LN2         1.44269502f
#define VCT_LOG2_C9         0.111111112f
#define VCT_LOG2_C7         0.142857149f
#define VCT_LOG2_C5         0.200000003f
#define VCT_LOG2_C3         0.333333343f

/* ---- diffuse cone sets ------------------------------------------------------
 * d_k = cn*n + ct*T + cb*B with (T,B) the Duff et al. 2017 branchless ONB of n.
 * Row = (cn, ct, cb, weight).  Weights are cos-theta normalised.               */
#define VCT_TAN30           0.577350259f /* 9-cone and 1-cone half-angle tangent   */
#define VCT_TAN20           0.36397022f  /* 16-cone half-angle tangent             */

/* 9 cones: d0 = n, d_k at 45 deg polar, phi_k = (k-1)*45 deg       */
#define VCT_CONES9(X)                                                   \
    X(1.0f,        0.0f,        0.0f,        0.150221109f)             \
    X(0.707106769f, 0.707106769f, 0.0f,      0.106222361f)             \
    X(0.707106769f, 0.5f,        0.5f,       0.106222361f)             \
    X(0.707106769f, 0.0f,        0.707106769f, 0.106222361f)           \
    X(0.707106769f, -0.5f,       0.5f,       0.106222361f)             \
    X(0.707106769f, -0.707106769f, 0.0f,     0.106222361f)             \
    X(0.707106769f, -0.5f,       -0.5f,      0.106222361f)             \
    X(0.707106769f, 0.0f,        -0.707106769f, 0.106222361f)          \
    X(0.707106769f, 0.5f,        -0.5f,      0.106222361f)

/* 1 cone (config C1): d0 = n, w = 1                                            */
#define VCT_CONES1(X)  X(1.0f, 0.0f, 0.0f, 1.0f)

/* 16 cones (config C5): centre + 5 at 30 deg + 10 at 60 deg (phi offset 18 deg) */
#define VCT_CONES16(X)                                                  \
    X(1.0f,        0.0f,          0.0f,          0.0968042314f)        \
    X(0.866025388f, 0.5f,          0.0f,          0.0838349238f)       \
    X(0.866025388f, 0.154508501f,  0.475528270f,  0.0838349238f)       \
    X(0.866025388f, -0.404508501f, 0.293892622f,  0.0838349238f)       \
    X(0.866025388f, -0.404508501f, -0.293892622f, 0.0838349238f)       \
    X(0.866025388f, 0.154508501f,  -0.475528270f, 0.0838349238f)       \
    X(0.5f,        0.823639095f,  0.267616570f,  0.0484021157f)        \
    X(0.5f,        0.509036958f,  0.700629294f,  0.0484021157f)        \
    X(0.5f,        0.0f,          0.866025388f,  0.0484021157f)        \
    X(0.5f,        -0.509036958f, 0.700629294f,  0.0484021157f)        \
    X(0.5f,        -0.823639095f, 0.267616570f,  0.0484021157f)        \
    X(0.5f,        -0.823639095f, -0.267616570f, 0.0484021157f)        \
    X(0.5f,        -0.509036958f, -0.700629294f, 0.0484021157f)        \
    X(0.5f,        0.0f,          -0.866025388f, 0.0484021157f)        \
    X(0.5f,        0.509036958f,  -0.700629294f, 0.0484021157f)        \
    X(0.5f,        0.823639095f,  -0.267616570f, 0.0484021157f)

#define VCT_MAX_CONES       17           /* 16 diffuse + 1 specular                */

/* ---- A.4 anisotropic faces --------------------------------------------------
 * Face f is the one SAMPLED by cones travelling along that direction; its
 * "front" child is the one a +X-travelling cone meets first (smaller x).      */
#define VCT_FACE_PX 0
#define VCT_FACE_NX 1
#define VCT_FACE_PY 2
#define VCT_FACE_NY 3
#define VCT_FACE_PZ 4
#define VCT_FACE_NZ 5
#define VCT_NUM_FACES 6

/* ---- A.2 voxelization fixed point ------------------------------------------ */
#define VCT_FIXED_ONE       65536.0f     /* round(x * 2^16) into int64 sums        */
#define VCT_FIXED_ONE_D     65536.0

/* ---- diffuse maps (albedo = Kd x diffuse map; SURVEY 8a Model::loadMaterials) --
 * The reference loads a material's map_Kd with stbi_load(path, .., 0), uploads it
 * as glTexImage2D(GL_RED | GL_RGB | GL_RGBA, GL_UNSIGNED_BYTE) and samples it with
 * GL_REPEAT wrap and GL_LINEAR magnification (model.cpp:150-226, :212-216) at the
 * assimp-flipped UV (aiProcess_FlipUVs, model.cpp:24: v' = 1 - v).
 *  Texture: W x H RGBA8, row 0 = the image's first (top) row = GL's t = 0 row;
 *    1 / 3 channels expand as GL_RED / GL_RGB sample: (r,0,0,255) / (r,g,b,255).
 *    (2 channels: the reference leaves `format` uninitialised, model.cpp:200-206;
 *    such a map is refused and the material keeps Kd.)
 *  Texel value c / 255.0f per channel (float division).
 *  T(u, v) for the TexCoords (u, v') of the vertex record (already flipped):
 *    fu = u - floorf(u), fv = v' - floorf(v')          (non-finite coordinate -> 0)
 *    s = fu * W - 0.5,  t = fv * H - 0.5               (texel-centre convention)
 *    x0 = floorf(s), ax = s - x0, x1 = x0 + 1 (likewise y0, ay, y1), wrapped into
 *    [0, W) / [0, H) (GL_REPEAT; x0 >= -1 and x1 <= W by construction)
 *    lerp(a, b, f) = fmaf(f, b - a, a)
 *    T = lerp(lerp(T[y0][x0], T[y0][x1], ax), lerp(T[y1][x0], T[y1][x1], ax), ay)
 *    rgb only.  Base level only: voxelization and the G-buffer have no screen-space
 *    derivative to pick a GL_LINEAR_MIPMAP_LINEAR level from.
 *  UV of a (triangle, voxel) hit in K1: the voxel centre c projected onto the
 *    triangle's plane, in voxel units (q0, q1, q2 = the vertices):
 *      e1 = q1 - q0, e2 = q2 - q0, w = c - q0, dot = (x*x' + y*y') + z*z'
 *      d11 = e1.e1, d12 = e1.e2, d22 = e2.e2, w1 = w.e1, w2 = w.e2
 *      den = d11*d22 - d12*d12; b1 = b2 = 0 unless den > 0, else
 *      b1 = (d22*w1 - d12*w2) / den, b2 = (d11*w2 - d12*w1) / den
 *      b1 = fmaxf(b1, 0), b2 = fmaxf(b2, 0); if (b1 + b2 > 1) b1 /= s, b2 /= s (s = b1 + b2)
 *    and in the G-buffer: (b1, b2) = the Moller-Trumbore (u, v) of the nearest hit.
 *    uv = fmaf(b2, uv2 - uv0, fmaf(b1, uv1 - uv0, uv0)) per component.
 *  Albedo = Kd.rgb * T.rgb, then (K1) round(albedo * 2^16) into the int64 sums. */
#define VCT_TEX_MAX_DIM     16384u       /* largest texture edge accepted           */

/* ---- multi-GPU screen tiling ---------------------------------- */
#define VCT_TILE            64           /* 64x64-pixel tiles, round-robin by rank */

/* Composite + present:
 *   direct = ((albedo * color) * max(n.l, 0)) * V     V: the K2 DDA shadow walk
 *            from q = (P - g0) * n/E + N (the cone origin) toward l
 *   final  = (direct + albedo * diffuse.rgb) + spec.rgb          (linear)
 *   rgba8  = round(255 * (f / (1 + f))^(1/2.2)) per channel, alpha 255;
 *            background pixels = the reference's clear colour
 *            (glClearColor(0.2, 0.3, 0.3, 1), r_voxelization.cpp:8). */
#define VCT_CLEAR_R         0.2f
#define VCT_CLEAR_G         0.3f
#define VCT_CLEAR_B         0.3f
#define VCT_INV_GAMMA       0.454545468f /* 1 / 2.2 */

#endif /* VCT_SPEC_H */
