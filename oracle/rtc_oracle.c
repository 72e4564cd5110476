/*
 * oracle/rtc_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement ("port") of the reference render
 * path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so, and
 * only as the checker / the timed CPU baseline -- never as the product path.
 *
 * It restates, in plain C with every float<->double promotion of the source kept explicit (SURVEY.md
 * Appendix A), the deterministic variant of the reference (per-pixel seed x + y*W reaching
 * the RNG, thread-local RNG state, run-time spp):
 *   vec3 math            moremath.c:7-87
 *   RNG                  moremath.c:89-108
 *   getEnvironmentLight  raytracing.c:151-160
 *   raySphere            raytracing.c:162-184
 *   rayTriangle          raytracing.c:186-214
 *   calculateRayCollision raytracing.c:216-240
 *   calcColor            raytracing.c:262-296
 *   calcDebugColor       raytracing.c:242-260 (RTC_F_DEBUG_BOUNCES)
 *   rowThread            main.c:81-104 (row-interleaved pthreads, main.c:84,285-302)
 *   vec3ToColor          raytracing.c:11-15 / moremath.c:25-30
 *
 * Pinned against oracle/_ref/rtc_ref (the reference's own sources built by oracle/Makefile) through the
 * golden fixtures in tests/golden/ (tests/test_oracle.py).  Compile with -ffp-contract=off and no
 * -ffast-math.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rtc.h"

#define ORC_EPS 0.001 /* scene.h:37, a double */

/* ---- moremath.c ------------------------------------------------------------------------------------ */
static inline float o_length(vec3 v) { return (float)sqrt((double)(v.x * v.x + v.y * v.y + v.z * v.z)); } /* :7-10 */
static inline vec3 o_normalized(vec3 v)                                                                     /* :12-17 */
{
    float invLen = (float)(1. / (double)o_length(v));
    vec3 r = {v.x * invLen, v.y * invLen, v.z * invLen};
    return r;
}
static inline float o_dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :33-36 */
static inline float o_clamp(float x) { return x < 0 ? 0 : (x > 1 ? 1 : x); }           /* :38-41 */
static inline vec3 o_cross(vec3 u, vec3 v)                                              /* :43-47 */
{
    vec3 r = {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
    return r;
}
static inline float o_smoothstep(float inf, float sup, float x) /* :49-53 */
{
    x = o_clamp((x - inf) / (sup - inf));
    return (float)((double)(x * x) * (3. - 2. * (double)x));
}
static inline vec3 o_plus(vec3 a, vec3 b) { vec3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static inline vec3 o_minus(vec3 a, vec3 b) { vec3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static inline vec3 o_times(vec3 a, float b) { vec3 r = {a.x * b, a.y * b, a.z * b}; return r; }
static inline vec3 o_timesVec3(vec3 a, vec3 b) { vec3 r = {a.x * b.x, a.y * b.y, a.z * b.z}; return r; }
static inline vec3 o_reflect(vec3 d, vec3 n) { return o_minus(d, o_times(n, (float)(2. * (double)o_dot(d, n)))); } /* :79-82 */
static inline vec3 o_lerp(vec3 a, vec3 b, float t) { return o_plus(o_times(a, 1 - t), o_times(b, t)); }              /* :84-87 */

static inline float o_random(unsigned int *s) /* :89-95 */
{
    *s = *s * 747796405u + 2891336453u;
    unsigned int r = ((*s >> ((*s >> 28) + 4)) ^ *s) * 277803737u;
    r = (r >> 22) ^ r;
    return (float)((double)r / 4294967295.0);
}
static inline float o_random_normal(unsigned int *s) /* :97-102 */
{
    float theta = (float)(2 * 3.14159265 * (double)o_random(s));
    float rho = (float)sqrt(-2 * log((double)o_random(s)));
    return (float)((double)rho * cos((double)theta));
}
static inline vec3 o_random_direction(unsigned int *s) /* :104-108; x, y, z drawn in that order */
{
    vec3 r;
    r.x = o_random_normal(s);
    r.y = o_random_normal(s);
    r.z = o_random_normal(s);
    return o_normalized(r);
}
static inline uint8 o_float_to_uint(float f) /* moremath.c:25-30; NaN -> 0 as cvttss2si on x86-64 */
{
    if (f < 0)
        return 0;
    if (f >= 1)
        return 255;
    if (f != f)
        return 0;
    return (uint8)(f * 255.f);
}

/* ---- raytracing.c ---------------------------------------------------------------------------------- */
static vec3 o_env(Ray ray, const Scene *s) /* :151-160 */
{
    float skyGradientT = powf(o_smoothstep(0.f, (float).74, -ray.dir.y), (float).35);
    vec3 skyGradient = o_lerp(s->skyColorHorizon, s->skyColorZenith, skyGradientT);
    float sun = powf((float)fmax(0., (double)o_dot(ray.dir, s->normalizedSunDirection)), s->sunFocus) * s->sunIntensity;
    float groundToSkyT = o_smoothstep((float)-0.01, 0.f, -ray.dir.y);
    float sunMask = ray.dir.y < 0;
    vec3 sunValue = {sun * sunMask, sun * sunMask, sun * sunMask};
    return o_plus(o_lerp(s->groundColor, skyGradient, groundToSkyT), sunValue);
}

typedef struct { int didHit; float dst; vec3 hitPoint; vec3 normal; Material mat; } OHit;

static OHit o_ray_sphere(Ray ray, vec3 c, float radius) /* :162-184 */
{
    OHit h;
    memset(&h, 0, sizeof h);
    vec3 offset = o_minus(ray.pos, c);
    float b = o_dot(offset, ray.dir);
    float cc = o_dot(offset, offset) - radius * radius;
    float delta = b * b - cc;
    if (delta < 0)
        return h;
    delta = (float)sqrt((double)delta);
    float dst = -b - delta;
    if ((double)dst < ORC_EPS)
        dst = -b + delta;
    if ((double)dst < ORC_EPS)
        return h;
    h.didHit = 1;
    h.dst = dst;
    h.hitPoint = o_plus(ray.pos, o_times(ray.dir, dst));
    h.normal = o_normalized(o_minus(h.hitPoint, c));
    return h;
}

static OHit o_ray_triangle(Ray ray, const Triangle *t) /* :186-214 */
{
    OHit h;
    memset(&h, 0, sizeof h);
    if (o_dot(ray.dir, t->normal) >= 0)
        return h;
    vec3 AB = o_minus(t->posB, t->posA);
    vec3 AC = o_minus(t->posC, t->posA);
    vec3 hh = o_cross(ray.dir, AC);
    float det = o_dot(AB, hh);
    if (-ORC_EPS < (double)det && (double)det < ORC_EPS)
        return h;
    float invDet = (float)(1. / (double)det);
    vec3 s = o_minus(ray.pos, t->posA);
    float u = o_dot(s, hh) * invDet;
    if (u < 0 || u > 1)
        return h;
    vec3 q = o_cross(s, AB);
    float v = o_dot(ray.dir, q) * invDet;
    if (v < 0 || u + v > 1)
        return h;
    float dst = o_dot(AC, q) * invDet;
    if ((double)dst < ORC_EPS)
        return h;
    h.dst = dst;
    h.didHit = 1;
    h.normal = t->normal;
    return h;
}

typedef struct {
    const Triangle *tris;
    int triCount;
    const Sphere *sph;
    int sphCount;
    const Scene *scene;
    int trianglesOnly;
    int maxBounce;
} OCtx;

static OHit o_collide(Ray ray, const OCtx *c, unsigned long long *segments) /* :216-240 */
{
    OHit closest;
    memset(&closest, 0, sizeof closest);
    closest.dst = 999999;
    (*segments)++;
    if (c->trianglesOnly == 0)
        for (int i = 0; i < c->sphCount; ++i) {
            OHit h = o_ray_sphere(ray, c->sph[i].pos, c->sph[i].r);
            if (h.didHit && h.dst < closest.dst) {
                closest = h;
                closest.mat = c->sph[i].mat;
            }
        }
    for (int i = 0; i < c->triCount; ++i) {
        OHit h = o_ray_triangle(ray, &c->tris[i]);
        if (h.didHit && h.dst < closest.dst) {
            closest = h;
            closest.mat = c->tris[i].mat;
        }
    }
    closest.hitPoint = o_plus(ray.pos, o_times(ray.dir, closest.dst));
    return closest;
}

static vec3 o_calc_color(Ray ray, const OCtx *c, unsigned int *rng, unsigned long long *segments) /* :262-296 */
{
    vec3 incomingLight = {0, 0, 0};
    vec3 rayColor = {1, 1, 1};
    for (int i = 0; i < c->maxBounce; ++i) {
        OHit hit = o_collide(ray, c, segments);
        if (hit.didHit) {
            vec3 diffuseDir = o_normalized(o_plus(hit.normal, o_random_direction(rng)));
            vec3 specularDir = o_reflect(ray.dir, hit.normal);
            ray.dir = o_lerp(diffuseDir, specularDir, hit.mat.smoothness);
            ray.pos = hit.hitPoint;
            vec3 emittedLight = o_times(hit.mat.color, hit.mat.emissionStrength);
            incomingLight = o_plus(incomingLight, o_timesVec3(emittedLight, rayColor));
            rayColor = o_timesVec3(rayColor, hit.mat.color);
            float p = (float)fmax(fmax((double)rayColor.x, (double)rayColor.y), (double)rayColor.z);
            if (p < o_random(rng))
                break;
            rayColor = o_times(rayColor, (float)(1.0 / (double)p));
        } else {
            incomingLight = o_plus(incomingLight, o_timesVec3(o_env(ray, c->scene), rayColor));
            break;
        }
    }
    return incomingLight;
}

/* calcDebugColor (raytracing.c:242-260): bounce count until the first miss, as grey */
static vec3 o_calc_debug_color(Ray ray, const OCtx *c, unsigned int *rng, unsigned long long *segments)
{
    int i;
    for (i = 0; i < c->maxBounce; ++i) {
        OHit hit = o_collide(ray, c, segments);
        if (hit.didHit) {
            vec3 diffuseDir = o_normalized(o_plus(hit.normal, o_random_direction(rng)));
            vec3 specularDir = o_reflect(ray.dir, hit.normal);
            ray.dir = o_lerp(diffuseDir, specularDir, hit.mat.smoothness);
            ray.pos = hit.hitPoint;
        } else
            break;
    }
    vec3 black = {0, 0, 0}, white = {1, 1, 1};
    return o_lerp(black, white, i / (float)c->maxBounce);
}

/* ---- rowThread (main.c:81-104) -------------------------------------------------------------------- */
typedef struct {
    const OCtx *ctx;
    const RtcCamera *cam;
    const RtcRenderDesc *d;
    int rows;
    int tid, nthreads;
    Color *out;
    float *accum;
    unsigned long long segments;
} OThread;

/* Launch row r -> image row y (rtc.h RtcRenderDesc): rows y = rowStart + k*rowStride (main.c:84's interleave), or with
 * rowBand B > 1 bands of B rows, band k starting at rowStart + k*rowStride*B */
static int oracle_row_y(const RtcRenderDesc *d, int r)
{
    const int B = d->rowBand > 1 ? d->rowBand : 1;
    return d->rowStart + (r / B) * d->rowStride * B + r % B;
}

static void *o_row_thread(void *p)
{
    OThread *a = p;
    const RtcRenderDesc *d = a->d;
    const int width = d->width, height = d->height;
    const float invSpp = (float)(1. / (double)d->spp);
    for (int r = a->tid; r < a->rows; r += a->nthreads) {
        int y = oracle_row_y(d, r);
        for (int x = 0; x < width; ++x) {
            float dx = (x - width / 2) / (float)(height / 2);
            float dy = (y - (height / 2)) / (float)(height / 2);
            vec3 dir = o_plus(o_plus(o_times(a->cam->ex, dx), o_times(a->cam->ey, dy)), o_times(a->cam->ez, a->cam->fov));
            dir = o_normalized(dir);
            Ray ray = {a->cam->origin, dir};
            unsigned int rng = (unsigned int)(x + y * width);
            vec3 acc = {0, 0, 0};
            for (int i = 0; i < d->spp; ++i) {
                vec3 c = (d->flags & RTC_F_DEBUG_BOUNCES) ? o_calc_debug_color(ray, a->ctx, &rng, &a->segments)
                                                         : o_calc_color(ray, a->ctx, &rng, &a->segments);
                acc = o_plus(acc, o_times(c, invSpp));
            }
            size_t o = (size_t)r * (size_t)width + (size_t)x;
            if (a->out) {
                a->out[o].r = o_float_to_uint(acc.x);
                a->out[o].g = o_float_to_uint(acc.y);
                a->out[o].b = o_float_to_uint(acc.z);
            }
            if (a->accum) {
                a->accum[3 * o] = acc.x;
                a->accum[3 * o + 1] = acc.y;
                a->accum[3 * o + 2] = acc.z;
            }
        }
    }
    return NULL;
}

/* ---- exported -------------------------------------------------------------------------------------- */
int oracle_rows_selected(const RtcRenderDesc *d)
{
    if (d->rowStride <= 0 || d->rowStart < 0 || d->rowStart >= d->height || d->rowBand < 0)
        return 0;
    const int B = d->rowBand > 1 ? d->rowBand : 1, step = d->rowStride * B;
    const int nb = (d->height - d->rowStart + step - 1) / step, last = d->rowStart + (nb - 1) * step;
    return (nb - 1) * B + (d->height - last < B ? d->height - last : B);
}

/* The render seam main.c:263-304 on the CPU: same arguments as rtc_render, plus the thread count. */
int oracle_render(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                  const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int nthreads,
                  Color *outImage, float *outAccum, unsigned long long *segments)
{
    if (!d || !cam || !scene || d->width <= 0 || d->height <= 0 || nthreads <= 0 || triCount < 0 ||
        (triCount > 0 && !tris) || (sphereCount > 0 && !spheres))
        return RTC_EINVAL;
    OCtx ctx = {tris, triCount, spheres, sphereCount, scene, d->trianglesOnly, d->maxBounce};
    int rows = oracle_rows_selected(d);
    OThread *ts = calloc((size_t)nthreads, sizeof(OThread));
    pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; ++i) {
        ts[i].ctx = &ctx;
        ts[i].cam = cam;
        ts[i].d = d;
        ts[i].rows = rows;
        ts[i].tid = i;
        ts[i].nthreads = nthreads;
        ts[i].out = outImage;
        ts[i].accum = outAccum;
        pthread_create(&th[i], NULL, o_row_thread, &ts[i]);
    }
    unsigned long long seg = 0;
    for (int i = 0; i < nthreads; ++i) {
        pthread_join(th[i], NULL);
        seg += ts[i].segments;
    }
    if (segments)
        *segments = seg;
    free(ts);
    free(th);
    return 0;
}

/* ---- single-function KAT entry points ------------------------------------------------------------- */
void oracle_ray_triangle(const Ray *rays, const Triangle *tris, size_t n, int *didHit, float *dst)
{
    for (size_t i = 0; i < n; ++i) {
        OHit h = o_ray_triangle(rays[i], &tris[i]);
        didHit[i] = h.didHit;
        dst[i] = h.dst;
    }
}

void oracle_ray_sphere(const Ray *rays, const Sphere *sph, size_t n, int *didHit, float *dst, vec3 *normal)
{
    for (size_t i = 0; i < n; ++i) {
        OHit h = o_ray_sphere(rays[i], sph[i].pos, sph[i].r);
        didHit[i] = h.didHit;
        dst[i] = h.dst;
        normal[i] = h.normal;
    }
}

void oracle_environment(const Ray *rays, const Scene *scenes, size_t n, vec3 *out)
{
    for (size_t i = 0; i < n; ++i)
        out[i] = o_env(rays[i], &scenes[i]);
}

void oracle_random(const unsigned int *seeds, size_t n, int draws, float *uniform, float *normal, vec3 *direction)
{
    for (size_t i = 0; i < n; ++i) {
        unsigned int s = seeds[i];
        for (int k = 0; k < draws; ++k)
            uniform[i * (size_t)draws + k] = o_random(&s);
        s = seeds[i];
        for (int k = 0; k < draws; ++k)
            normal[i * (size_t)draws + k] = o_random_normal(&s);
        s = seeds[i];
        for (int k = 0; k < draws; ++k)
            direction[i * (size_t)draws + k] = o_random_direction(&s);
    }
}

/* calcColor on explicit rays/seeds (tests compare with the reference's own calcColor via rtc_ref --kat-calc) */
void oracle_calc_color(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                       const Scene *scene, int trianglesOnly, const Ray *rays, const unsigned int *seeds,
                       const int *maxBounce, size_t n, vec3 *out, unsigned int *seedAfter, int debug)
{
    for (size_t i = 0; i < n; ++i) {
        OCtx ctx = {tris, triCount, spheres, sphereCount, scene, trianglesOnly, maxBounce[i]};
        unsigned int s = seeds[i];
        unsigned long long seg = 0;
        out[i] = debug ? o_calc_debug_color(rays[i], &ctx, &s, &seg) : o_calc_color(rays[i], &ctx, &s, &seg);
        seedAfter[i] = s;
    }
}
