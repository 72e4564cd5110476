/*
 * rtc_device.h -- device-side restatement of the reference math for gfx950.
 *
 * Every function follows the reference expression by expression, with the reference's float<->double
 * promotions.  The translation unit is compiled with -ffp-contract=off and
 * without fast-math: a fused multiply-add changes Monte-Carlo paths.  f32 division is the
 * IEEE one (hipcc default -fhip-fp32-correctly-rounded-divide-sqrt); a double divide rounded to float
 * equals the f32 IEEE divide (double rounding is innocuous for 53 >= 2*24+2), so `(float)(1./x)` in
 * the source is `1.f / x` here.
 */
#pragma once
#include <hip/hip_runtime.h>

/* Timing-experiment switches that change the frame (not the reference's arithmetic): a build defines one only together
 * with RTC_EXPERIMENT, which the Makefile's product targets never define. */
#if (defined(RTC_AB_CHEAP_ENV_SKY) || defined(RTC_AB_CHEAP_DIR) || defined(RTC_AB_NO_SLOTS)) && !defined(RTC_EXPERIMENT)
#error "RTC_AB_* switches produce a wrong frame (timing experiments only): define RTC_EXPERIMENT as well"
#endif

#include "rtc_math.h"

namespace rtcdev {

struct V3 {
    float x, y, z;
};

__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }      /* moremath.c:55-59 */
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }      /* :61-65 */
__device__ __forceinline__ V3 mul(V3 a, float b) { return V3{a.x * b, a.y * b, a.z * b}; }         /* :67-71 */
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }     /* :73-77 */
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }     /* :33-36 */
__device__ __forceinline__ V3 cross(V3 u, V3 v)                                                    /* :43-47 */
{
    return V3{u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
/* Correctly rounded f32 sqrt.  The reference's sqrt of a float in double, rounded to float, is the same
 * value (double rounding is innocuous for sqrt: 53 >= 2*24+2); llvm.sqrt.f32 is correctly rounded under
 * HIP's default -fhip-fp32-correctly-rounded-divide-sqrt.  Checked for all 2^32 inputs
 * (tools/exact_probe.hip, tests/test_gpu_exact.py). */
__device__ __forceinline__ float sqrt_cr(float x) { return __builtin_sqrtf(x); }

/* Correctly rounded 1/x, == the IEEE f32 divide 1.f / x (and so == (float)(1./x)).  For |x| in
 * [2^-125, 2^125]: v_rcp_f32 (<= 1 ulp) and two FMA Newton steps (the residual 1 - x r is exact in an FMA when
 * r is within an ulp; the second step leaves an error far below the distance of 1/x from any rounding
 * midpoint); other x take the divide.  Checked for all 2^32 inputs (tools/exact_probe.hip). */
__device__ __forceinline__ float rcp_cr(float x)
{
    const float ax = __builtin_fabsf(x);
    if (ax >= 0x1p-125f && ax <= 0x1p125f) {
        float r = __builtin_amdgcn_rcpf(x);
        r = __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
    return 1.f / x;
}

/* length (moremath.c:7-10): sqrt of the f32 sum in double, rounded to float (== correctly rounded sqrtf) */
__device__ __forceinline__ float length(V3 v) { return sqrt_cr(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ V3 normalized(V3 v) /* :12-17 */
{
    float invLen = rcp_cr(length(v)); /* (float)(1./length(v)) */
    return V3{v.x * invLen, v.y * invLen, v.z * invLen};
}
__device__ __forceinline__ float clamp01(float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); } /* :38-41 */
__device__ __forceinline__ float smoothstep(float inf, float sup, float x)                          /* :49-53 */
{
    x = clamp01((x - inf) / (sup - inf));
    return (float)((double)(x * x) * (3.0 - 2.0 * (double)x));
}
/* getEnvironmentLight's two smoothsteps (raytracing.c:153 smoothstep(0, .74f, -dir.y), :156
 * smoothstep(-.01f, 0, -dir.y)) with the f32 divide by the constant sup - inf done as a multiply by its
 * rounded reciprocal plus one FMA remainder correction (q = n rd, r = n - q d exactly, q + r rd), which is the
 * correctly rounded n / d here.  n is first limited to [-2, 2] (NaN kept): beyond that the quotient clamps to
 * the same 0 or 1, and the product cannot overflow.  Bit-identical to smoothstep() for all 2^32 x
 * (tools/exact_probe.hip). */
constexpr int kSkyStep = 0, kGroundStep = 1;
template <int S> __device__ __forceinline__ float smoothstep_k(float x)
{
    constexpr float inf = S == kSkyStep ? 0.f : -0.01f;
    constexpr float sup = S == kSkyStep ? 0.74f : 0.f;
    constexpr float d = sup - inf;
    constexpr float rd = 1.f / d;
    float n = x - inf;
    n = n > 2.f ? 2.f : n;
    n = n < -2.f ? -2.f : n;
    const float q = n * rd;
    x = clamp01(fmaf(fmaf(-q, d, n), rd, q));
    return (float)((double)(x * x) * (3.0 - 2.0 * (double)x));
}
__device__ __forceinline__ V3 reflect(V3 d, V3 n) { return sub(d, mul(n, 2.f * dot(d, n))); }  /* :79-82; 2*f exact */
__device__ __forceinline__ V3 lerp(V3 a, V3 b, float t) { return add(mul(a, 1.f - t), mul(b, t)); } /* :84-87 */

/* RandomValue (moremath.c:89-95) on a register-resident per-pixel state */
__device__ __forceinline__ float random_value(unsigned &s)
{
    s = s * 747796405u + 2891336453u;
    unsigned r = ((s >> ((s >> 28) + 4)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    /* (float)((double)r / 4294967295.0) without the double divide: r/(2^32-1) = r 2^-32 (1 + 2^-32 + ...)
     * lies within r 2^-64 (< 2^-32) above r 2^-32, which cannot reach the next float rounding boundary but
     * does push an exact tie upward; r 2^-32 + r 2^-64 (one rounding) does the same.  Equal for all 2^32
     * values of r (checked exhaustively, tools/check_devmath.cpp). */
    const double d = (double)r * 0x1p-32;
    return (float)fma((double)r, 0x1p-64, d);
}
/* The LCG step of RandomValue is affine mod 2^32, so k steps are one: s_k = A_k s + C_k with A_k = a^k and
 * C_k = c (a^(k-1) + ... + 1).  rng_jump_value(s, k) is the value of the k-th draw from state s (k >= 1),
 * i.e. what k calls of random_value would return last; it does not advance s. */
struct RngJump {
    unsigned a, c;
};
constexpr RngJump rng_jump(int k)
{
    unsigned A = 1u, C = 0u;
    for (int i = 0; i < k; ++i) {
        C = C * 747796405u + 2891336453u;
        A = A * 747796405u;
    }
    return RngJump{A, C};
}
/* jump by any k draws: compose the power-of-two jumps of k's set bits */
constexpr RngJump rng_compose(RngJump x, RngJump y) { return RngJump{x.a * y.a, x.c * y.a + y.c}; } /* x then y */
struct RngPow2Table {
    RngJump j[32];
    constexpr RngPow2Table() : j{}
    {
        j[0] = rng_jump(1);
        for (int b = 1; b < 32; ++b)
            j[b] = rng_compose(j[b - 1], j[b - 1]);
    }
};
__device__ __forceinline__ unsigned rng_advance(unsigned s, unsigned k)
{
    constexpr RngPow2Table T;
    for (int b = 0; b < 32 && (k >> b) != 0u; ++b)
        if ((k >> b) & 1u)
            s = s * T.j[b].a + T.j[b].c;
    return s;
}
/* the affine map of k draws as (a, c): rng_advance(s, k) == s * a + c */
__device__ __forceinline__ RngJump rng_jump_by(unsigned k)
{
    constexpr RngPow2Table T;
    RngJump j{1u, 0u};
    for (int b = 0; b < 32 && (k >> b) != 0u; ++b)
        if ((k >> b) & 1u)
            j = rng_compose(j, T.j[b]);
    return j;
}
__device__ __forceinline__ float rng_value_of_state(unsigned s)
{
    unsigned r = ((s >> ((s >> 28) + 4)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    const double d = (double)r * 0x1p-32;
    return (float)fma((double)r, 0x1p-64, d);
}

/* RandomValueNormalDistrubtion (moremath.c:97-102): Box-Muller cos branch in double */
__device__ __forceinline__ float random_normal(unsigned &s)
{
    float theta = (float)(2 * 3.14159265 * (double)random_value(s));
    float rho = (float)__builtin_sqrt(-2 * rtcmath::log((double)random_value(s)));
    return (float)((double)rho * rtcmath::cos((double)theta));
}
/* the exact restatement of three normals (the fallback of random_direction); inlined (out of line the chain kernel
 * spilled less but ran ~1.5% slower; one normal at a time in a loop, no gain: round 4) */
static __device__ __forceinline__ void random_normals_exact(unsigned &s, float v[3])
{
    v[0] = random_normal(s);
    v[1] = random_normal(s);
    v[2] = random_normal(s);
}
/* RandomDiretion (moremath.c:104-108), components drawn x, y, z.  The three normals take the certified fast
 * path (rtc_math.h bm_rho_fast / bm_normal_fast: table-driven log and cos, each float returned only when it
 * provably rounds like the reference's); a lane with any uncertified value (~4e-6 per normal) redraws all three
 * from the saved state with the exact restatement (random_normal). */
__device__ __forceinline__ V3 random_direction(unsigned &s, const rtcmath::BmLogEntry *logTab = rtcmath::kBmLogTab,
                                              const double (*cosTab)[2] = rtcmath::kBmCosTab)
{
#ifdef RTC_AB_CHEAP_DIR /* timing experiment only (the Box-Muller cost): six draws, no log / cos -- not the reference */
    const float a = random_value(s) - .5f, b = random_value(s) - .5f, c = random_value(s) - .5f;
    (void)random_value(s), (void)random_value(s), (void)random_value(s);
    return normalized(V3{a, b, c + 1e-3f});
#endif
    const unsigned s0 = s;
    float v[3];
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float theta = (float)(2 * 3.14159265 * (double)random_value(s)); /* moremath.c:99 */
        float rho;
        ok = rtcmath::bm_rho_fast(random_value(s), rho, logTab) && ok;
        ok = rtcmath::bm_normal_fast(rho, theta, v[c], cosTab) && ok;
    }
    if (__builtin_expect(!ok, 0)) {
#ifdef RTC_DIAG /* diagnostic builds: the lanes that take the fallback, per wave slot (rtc_diag_itemlog) */
        atomicAdd(&g_rtc_bmfall[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & 65535u], 1u);
#endif
        s = s0;
        random_normals_exact(s, v);
    }
    return normalized(V3{v[0], v[1], v[2]});
}

/* powf for the environment (raytracing.c:153,155): glibc 2.35's own powf algorithm, tables and
 * coefficients, as its x86-64 FMA build evaluates it (rtc_math.h powf_glibc): bit-identical to the
 * reference's powf calls (tools/check_devmath.cpp: every float x in [0, 1] for the exponents checked). */
struct EnvParams {
    V3 sun, horizon, zenith, ground;
    float focus, intensity;
    bool sunSkip; /* env_sun_skippable(focus, intensity) */
    /* sun_vanishes' limit on focus * log2(x) (env_vanish_limit; -inf: never) */
    double vanishLim;
    /* powf tables: every kernel that evaluates the environment points them at its LDS copies (PowTablesLds; round 4:
     * no null-table branch to glibc's constants in global memory, whose code the sky kernel paid for in spills) */
    const double (*log2tab)[2];
    const unsigned long long *exp2tab;
};

/* the sun term's powf (raytracing.c:155).  Its x = fmax0_ref(.) is +0 .. +inf or -0, never NaN or negative.  With y
 * not special (a launch constant: a wave-uniform branch) glibc's positive-x path gives powf(|x|, y), and powf(-0, y)
 * is powf(+0, y) with the sign of x when y is an odd integer (e_powf.c: x2 = x * x, negated for odd y; 1 / x2 for
 * y < 0); a special y (+-0, +-inf, NaN) has e_powf.c's short list of results.  No lane takes a divergent general
 * path: round 4 replaced a per-lane branch to the whole of powf_glibc (taken for x = -0), whose code the sky and
 * chain kernels carried (frame 0.349 -> 0.344 ms, sky kernel -2.5 %). */
__device__ __forceinline__ float pow_ref(float x, float y, const EnvParams &s)
{
    const unsigned iy = rtcmath::f2u(y);
    if (!rtcmath::powf_zeroinfnan(iy)) {
        const float ax = __builtin_fabsf(x);
        const float r = rtcmath::powf_glibc_pos<true>(ax, y, s.log2tab, s.exp2tab);
        const bool odd = rtcmath::powf_checkint(iy) == 1; /* uniform */
        return (odd && rtcmath::f2u(x) == 0x80000000u) ? -r : r;
    }
    return rtcmath::powf_special_y(x, y);
}

/* The powf tables staged in LDS by a workgroup (call before its first __syncthreads) */
struct PowTablesLds {
    double log2tab[16][2];
    unsigned long long exp2tab[32];
    __device__ __forceinline__ void fill(int tid)
    {
        if (tid < 32)
            log2tab[tid >> 1][tid & 1] = rtcmath::powf_data::kLog2Tab[tid >> 1][tid & 1];
        else if (tid < 64)
            exp2tab[tid - 32] = rtcmath::powf_data::kExp2Tab[tid - 32];
    }
    __device__ __forceinline__ void attach(EnvParams &e) const
    {
        e.log2tab = log2tab;
        e.exp2tab = exp2tab;
    }
};

/* getEnvironmentLight (raytracing.c:151-160) */
/* fmax(0, v) as the reference's libm evaluates it (raytracing.c:155, double fmax of a float): NaN -> 0, v < 0
 * -> +0, otherwise v itself -- -0 included (x86-64 glibc returns its second operand for equal zeros) */
__device__ __forceinline__ float fmax0_ref(float v) { return (v < 0.f || v != v) ? 0.f : v; }
/* fmax(x, y) likewise (raytracing.c:283, Russian roulette): x > y ? x : y, the other operand when one is NaN;
 * y for equal values (the sign of equal zeros) */
__device__ __forceinline__ float fmax_ref(float x, float y) { return (x > y || y != y) ? x : y; }

/* Whether getEnvironmentLight's sun term sun * sunMask (raytracing.c:155-158) is known without its powf when
 * x = fmax(0, dot(dir, sunDir)) is +0 or the mask is 0 with x <= 1 (x not -0): with focus > 0, powf(x, focus)
 * is then a finite value >= +0 (+0 for x = +0, <= 1 for x <= 1), and with a finite intensity the product is a
 * zero of intensity's sign. */
__host__ __device__ __forceinline__ bool env_sun_skippable(float focus, float intensity)
{
    return focus > 0.f && intensity - intensity == 0.f; /* focus > 0, intensity finite */
}

/* getEnvironmentLight (raytracing.c:151-160).  A powf whose value is known for every live lane of the wave is
 * not evaluated (a wave-uniform branch, values unchanged): skyGradientT when smoothstep gives +0 (powf(+0, .35)
 * = +0) -- rays below the horizon --, the sun term as env_sun_skippable says. */
/* Round 6: the sun term provably adds nothing to any colour component.  With every component of the ground, horizon and
 * zenith colours >= m > 0, each component of lerp(ground, lerp(horizon, zenith, a), b) = g (1 - b) + s b (a, b in [0, 1];
 * fl(1 - b) >= (1 - b)(1 - u), each product and sum rounded) is >= m (1 - u)^6, so its exponent is at least
 * E = floor(log2(m (1 - 2^-20))) and the spacing above it at least 2^(E - 23): with H = 2^(E - 24), a sun term
 * 0 <= sv < H leaves every component's sum e + sv == e (round to nearest).  sv = fl(powf(x, focus) * intensity) for
 * sunMask = 1, and glibc's powf is exp2 of the double ylogx = focus * log2(x) it computes (powf_log2 and the same product:
 * the bits sun_vanishes compares) with a relative error below 2^-23 (its exp2 polynomial ~2^-30, the float rounding
 * 2^-24); with the product's rounding sv <= 2^ylogx * intensity * (1 + 2^-22).  So ylogx < log2(H / intensity) - 1e-5
 * (env_vanish_limit, on the host in double) proves sv < H.  Required: focus > 0 and finite (sunSkip), intensity > 0 and
 * finite, x a normal float in (0, 1), every colour component in [2^-60, 2^60] (no product underflows or overflows; else
 * the limit is -inf).  Skipping the powf then is the sunKnown skip of a value known to vanish (tests/test_gpu_parity.py
 * whole frames, tests/test_oracle_env.py the bound against the oracle's environment on every tested direction). */
__host__ __device__ inline double env_vanish_limit(float focus, float intensity, const float col[9])
{
    if (!(focus > 0.f) || !(intensity > 0.f) || !(focus < 3.0e38f) || !(intensity < 3.0e38f))
        return -__builtin_inf();
    double m = 1e300;
    for (int i = 0; i < 9; ++i) {
        if (!(col[i] >= 0x1p-60f) || !(col[i] <= 0x1p60f))
            return -__builtin_inf();
        m = col[i] < m ? (double)col[i] : m;
    }
    int E = 0;
    (void)frexp(m * (1.0 - 0x1p-20), &E); /* m (1 - 2^-20) = f 2^E, f in [0.5, 1): floor(log2) = E - 1 */
    const double H = ldexp(1.0, (E - 1) - 24);
    return log2(H / (double)intensity) - 1e-5;
}
__device__ __forceinline__ bool sun_vanishes(V3 dir, const EnvParams &s)
{
    const float x = fmax0_ref(dot(dir, s.sun));
    const unsigned ix = __float_as_uint(x);
    if (!(s.vanishLim > -1e300) || !(dir.y < 0.f) || ix < 0x00800000u || ix >= 0x3f800000u)
        return false;
    const double ylogx = (double)s.focus * rtcmath::powf_log2<true>(ix, s.log2tab);
    return ylogx < s.vanishLim;
}

template <bool kMissTerm>
__device__ __forceinline__ V3 environment_t(V3 dir, const EnvParams &s, bool sunVanish = false)
{
    const float skyArg = smoothstep_k<kSkyStep>(-dir.y);
    float skyGradientT = 0.f;
    /* smoothstep's value is +0 .. 1 or NaN (never negative, never -0: clamp01 keeps -0 but (-0)^2 = +0) and the
     * exponent 0.35 is not special, so glibc's powf takes its positive-x path: that path alone, branch-free */
    const unsigned sa = __float_as_uint(skyArg);
    if (__all(sa - 0x00800000u <= 0x3f800000u - 0x00800000u)) /* every lane normal x in (0, 1]: main path */
        skyGradientT = rtcmath::powf_sky_unit(skyArg, s.log2tab, s.exp2tab);
    else if (__any(sa != 0u))
        skyGradientT = rtcmath::powf_glibc_pos<true>(skyArg, 0.35f, s.log2tab, s.exp2tab);
    V3 skyGradient = lerp(s.horizon, s.zenith, skyGradientT);
    const float sunArg = fmax0_ref(dot(dir, s.sun));
    float groundToSkyT = smoothstep_k<kGroundStep>(-dir.y);
    float sunMask = dir.y < 0.f ? 1.f : 0.f;
    float sv = __builtin_copysignf(0.f, s.intensity);
    const bool sunKnown = (s.sunSkip && __float_as_uint(sunArg) != 0x80000000u && /* powf(-0, odd) = -0 */
                           (sunArg == 0.f || (sunMask == 0.f && sunArg <= 1.f))) ||
                          sunVanish;
    if (__any(!sunKnown)) {
        const float sun = pow_ref(sunArg, s.focus, s) * s.intensity;
        sv = sun * sunMask;
    } else if (kMissTerm) {
        return lerp(s.ground, skyGradient, groundToSkyT); /* sv is a zero: see environment_miss_term */
    }
    const V3 e = add(lerp(s.ground, skyGradient, groundToSkyT), V3{sv, sv, sv});
    return kMissTerm ? add(V3{0.f, 0.f, 0.f}, e) : e;
}
__device__ __forceinline__ V3 environment(V3 dir, const EnvParams &s) { return environment_t<false>(dir, s); }
/* A camera ray's miss as main.c:97-99 accumulates it: the sample is calcColor's light = 0 + environment * (1, 1, 1)
 * (raytracing.c:289-291), added to the pixel's sum as sum + sample * (1 / spp).  This returns a value m with
 * sum + m * (1/spp) == sum + (0 + e) * (1/spp) for every sum that is not -0 -- a sum that starts at +0 and only adds such
 * terms never is (x + y = -0 needs x = y = -0 in round-to-nearest): with the sun term known to be a zero (sv = +-0,
 * every lane of the wave) e = x + sv, and m = x.  For x not a zero, x + sv = x and 0 + x = x; for x = +-0 the term
 * is +-0 either way and sum + (+-0) = sum; a NaN x passes through both adds unchanged.  So the two adds by zero per
 * component are not executed: the reference's values, bit for bit, with 6 fewer VALU operations per sky sample.
 * Otherwise (a sun term computed) m = 0 + e, the reference's operations as they are. */
__device__ __forceinline__ V3 environment_miss_term(V3 dir, const EnvParams &s, bool sunVanish = false)
{
    return environment_t<true>(dir, s, sunVanish);
}

/* EPSILON is the double 0.001 (scene.h:37); for any float v, v < 0.001 <=> v < 0.001f and
 * -0.001 < v <=> -0.001f < v, so the float compares below are exact restatements. */
constexpr float kEps = 0.001f;

/* rayTriangle (raytracing.c:186-214) with the edges AB = B-A, AC = C-A precomputed (the same f32
 * subtraction the reference performs per call).  Returns dst if hit, else a negative sentinel. */
__device__ __forceinline__ bool ray_triangle(V3 pos, V3 dir, V3 A, V3 AB, V3 AC, V3 N, float &dstOut)
{
    if (dot(dir, N) >= 0.f)
        return false;
    V3 h = cross(dir, AC);
    float det = dot(AB, h);
    if (-kEps < det && det < kEps)
        return false;
    float invDet = rcp_cr(det); /* IEEE 1.f / det */
    V3 s = sub(pos, A);
    float u = dot(s, h) * invDet;
    if (u < 0.f || u > 1.f)
        return false;
    V3 q = cross(s, AB);
    float v = dot(dir, q) * invDet;
    if (v < 0.f || u + v > 1.f)
        return false;
    float dst = dot(AC, q) * invDet;
    if (dst < kEps)
        return false;
    dstOut = dst;
    return true;
}

/* raySphere (raytracing.c:162-184) -- distance only; the normal is formed by the caller when this
 * sphere wins (it is a function of the same hitPoint = pos + dir*dst). */
__device__ __forceinline__ bool ray_sphere(V3 pos, V3 dir, V3 c, float radius, float &dstOut)
{
    V3 offset = sub(pos, c);
    float b = dot(offset, dir);
    float cc = dot(offset, offset) - radius * radius;
    float delta = b * b - cc;
    if (delta < 0.f)
        return false;
    delta = (float)__builtin_sqrt((double)delta);
    float dst = -b - delta;
    if (dst < kEps)
        dst = -b + delta;
    if (dst < kEps)
        return false;
    dstOut = dst;
    return true;
}

/* floatToUint (moremath.c:25-30); NaN -> 0 like the x86-64 build of the reference */
__device__ __forceinline__ unsigned char float_to_u8(float f)
{
    if (f < 0.f)
        return 0;
    if (f >= 1.f)
        return 255;
    if (f != f)
        return 0;
    return (unsigned char)(unsigned)(f * 255.f);
}

} // namespace rtcdev
