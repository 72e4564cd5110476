/*
 * scene_build.c -- host scene build, the stage in front of the render path (SURVEY.md §8 f #1).
 *
 * Restates, with identical results on well-formed inputs, the reference's
 *   loadObj / loadMtl           objloader.c:221-551  (OBJ `v`, `vn`, `f a/b/c x3`, `mtllib`, `usemtl`;
 *                                                     MTL `newmtl`, `Kd`, `Ke`, `Ns`)
 *   loadOBJTriangles            raytracing.c:100-147 (x,y negation = "rotateZ 180deg")
 *   cleanFile/parseTriangleFile raytracing.c:19-98   (triangles.txt)
 * plus the scene defaults of scene.h:17-19 and main.c:14,21-28, the camera basis of main.c:252-255 and a
 * BMP writer byte-identical to stbi_write_bmp (stbi_image_write.h:451-529).
 *
 * Quirks kept on purpose (they decide the Triangle[] bytes): the face normal is the `vn` of the FIRST face
 * vertex (objloader.c:499); quads keep their first three vertices; an unknown / absent material gives
 * white, emission 0, smoothness 0 (objloader.c:501-506); Ns -> sqrt(0.001*Ns) (objloader.c:272); a second
 * `mtllib` line is appended to the first one's path (objloader.c:406); lines are matched by prefix at
 * column 0, and "\n"-only or '#' lines are skipped.
 * Where the reference has undefined behaviour (uninitialised malloc'd fields, out-of-range indices,
 * face lines that only partly match `a/b/c`), this code uses zeros and returns no error; documented in
 * DESIGN.md.  Nothing here calls exit().
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtc.h"
#include "rtc_internal.h"

/* ---- reference float math used by the host stage (moremath.c:7-47; gcc, no FMA contraction) -------- */
static vec3 h_sub(vec3 a, vec3 b) { vec3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static vec3 h_cross(vec3 u, vec3 v)
{
    vec3 r = {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
    return r;
}
static vec3 h_normalized(vec3 v)
{
    float len = (float)sqrt((double)(v.x * v.x + v.y * v.y + v.z * v.z));
    float inv = (float)(1. / (double)len);
    vec3 r = {v.x * inv, v.y * inv, v.z * inv};
    return r;
}

/* ---- growable arrays ------------------------------------------------------------------------------- */
typedef struct { void *p; size_t n, cap, elt; } Vec;
static int vec_push(Vec *v, const void *e)
{
    if (v->n == v->cap) {
        size_t nc = v->cap ? v->cap * 2 : 64;
        void *np = realloc(v->p, nc * v->elt);
        if (!np)
            return RTC_ENOMEM;
        v->p = np;
        v->cap = nc;
    }
    memcpy((char *)v->p + v->n * v->elt, e, v->elt);
    v->n++;
    return 0;
}

typedef struct { char name[128]; vec3 color; float emission, smoothness; } MtlEntry;

/* loadMtl (objloader.c:221-313) into `mats`; 1 if the file cannot be opened (a warning, not an error) */
static int read_mtl(const char *path, Vec *mats)
{
    FILE *fp = fopen(path, "r");
    if (!fp)
        return 1;
    mats->n = 0;
    char *line = NULL;
    size_t cap = 0;
    ssize_t len;
    MtlEntry *cur = NULL;
    while ((len = getline(&line, &cap, fp)) != -1) {
        if (len == 1 || line[0] == '#')
            continue;
        if (strncmp(line, "newmtl ", 7) == 0) {
            MtlEntry m;
            memset(&m, 0, sizeof m);
            char nm[256];
            if (sscanf(line, "newmtl %255s", nm) == 1) {
                snprintf(m.name, sizeof m.name, "%.127s", nm);
                if (vec_push(mats, &m) != 0)
                    break;
                cur = (MtlEntry *)mats->p + (mats->n - 1);
            }
        }
        if (!cur)
            continue;
        if (strncmp(line, "Ns ", 3) == 0) {
            float ns;
            if (sscanf(line, "Ns %f", &ns) == 1)
                cur->smoothness = (float)sqrt(0.001 * (double)ns);
        } else if (strncmp(line, "Kd ", 3) == 0) {
            sscanf(line, "Kd %f %f %f", &cur->color.x, &cur->color.y, &cur->color.z);
        } else if (strncmp(line, "Ke ", 3) == 0) {
            float g, b;
            sscanf(line, "Ke %f %f %f", &cur->emission, &g, &b);
        }
    }
    free(line);
    fclose(fp);
    return 0;
}

int rtc_load_obj(const char *path, Triangle **outTris, int *outCount)
{
    if (!path || !outTris || !outCount)
        return rtc_fail(RTC_EINVAL, "rtc_load_obj: null argument");
    *outTris = NULL;
    *outCount = 0;
    FILE *fp = fopen(path, "r");
    if (!fp)
        return rtc_fail(RTC_EIO, "ERROR WHILE LOADING OBJ ! (%s)", path);

    /* material library paths are resolved against the OBJ's directory (objloader.c:343-345) */
    char mtlPath[1024];
    const char *slash = strrchr(path, '/');
    if (slash)
        snprintf(mtlPath, sizeof mtlPath, "%.*s/", (int)(slash - path), path);
    else
        snprintf(mtlPath, sizeof mtlPath, "./");
    if (slash == path)
        snprintf(mtlPath, sizeof mtlPath, "/");

    Vec verts = {NULL, 0, 0, sizeof(vec3)}, norms = {NULL, 0, 0, sizeof(vec3)};
    Vec mats = {NULL, 0, 0, sizeof(MtlEntry)}, tris = {NULL, 0, 0, sizeof(Triangle)};
    const vec3 zero = {0, 0, 0};
    /* OBJ indices are 1-based: slot 0 is a placeholder, as in the reference's max+1 arrays */
    vec_push(&verts, &zero);
    vec_push(&norms, &zero);
    int currentMtl = -1;
    int rc = 0;
    char *line = NULL;
    size_t cap = 0;
    ssize_t len;
    while ((len = getline(&line, &cap, fp)) != -1) {
        if (len == 1 || line[0] == '#')
            continue;
        char word[256];
        if (strncmp(line, "mtllib ", 7) == 0) {
            if (sscanf(line, "mtllib %255s", word) == 1) {
                strncat(mtlPath, word, sizeof mtlPath - strlen(mtlPath) - 1);
                if (read_mtl(mtlPath, &mats) != 0)
                    rtc_log(1, "WARNING: No material found.\n");
            }
        } else if (strncmp(line, "usemtl ", 7) == 0) {
            if (sscanf(line, "usemtl %255s", word) == 1) {
                currentMtl = -1;
                for (size_t i = 0; i < mats.n; ++i)
                    if (strcmp(word, ((MtlEntry *)mats.p)[i].name) == 0) {
                        currentMtl = (int)i;
                        break;
                    }
            }
        } else if (strncmp(line, "v ", 2) == 0) {
            vec3 v = zero;
            sscanf(line, "v %f %f %f", &v.x, &v.y, &v.z);
            if ((rc = vec_push(&verts, &v)) != 0)
                break;
        } else if (strncmp(line, "vn ", 3) == 0) {
            vec3 v = zero;
            sscanf(line, "vn %f %f %f", &v.x, &v.y, &v.z);
            if ((rc = vec_push(&norms, &v)) != 0)
                break;
        } else if (strncmp(line, "f ", 2) == 0) {
            int ix[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            sscanf(line, "f %d/%d/%d %d/%d/%d %d/%d/%d", &ix[0], &ix[1], &ix[2], &ix[3], &ix[4], &ix[5], &ix[6],
                   &ix[7], &ix[8]);
            const vec3 *V = verts.p, *N = norms.p;
#define VAT(i) (((i) > 0 && (size_t)(i) < verts.n) ? V[(i)] : zero)
#define NAT(i) (((i) > 0 && (size_t)(i) < norms.n) ? N[(i)] : zero)
            vec3 a = VAT(ix[0]), b = VAT(ix[3]), c = VAT(ix[6]), n = NAT(ix[2]);
#undef VAT
#undef NAT
            Triangle t;
            /* loadOBJTriangles (raytracing.c:123-141): x and y negated, z kept */
            t.posA = (vec3){-a.x, -a.y, a.z};
            t.posB = (vec3){-b.x, -b.y, b.z};
            t.posC = (vec3){-c.x, -c.y, c.z};
            t.normal = (vec3){-n.x, -n.y, n.z};
            if (currentMtl < 0 || (size_t)currentMtl >= mats.n) {
                t.mat.color = (vec3){1.f, 1.f, 1.f};
                t.mat.emissionStrength = 0;
                t.mat.smoothness = 0;
            } else {
                const MtlEntry *m = (const MtlEntry *)mats.p + currentMtl;
                t.mat.color = m->color;
                t.mat.emissionStrength = m->emission;
                t.mat.smoothness = m->smoothness;
            }
            if ((rc = vec_push(&tris, &t)) != 0)
                break;
        }
    }
    free(line);
    fclose(fp);
    free(verts.p);
    free(norms.p);
    free(mats.p);
    if (rc != 0) {
        free(tris.p);
        return rtc_fail(rc, "rtc_load_obj: out of memory");
    }
    *outTris = tris.p;
    *outCount = (int)tris.n;
    return 0;
}

/* cleanFile (raytracing.c:47-74): keep [0-9.+-\n], drop `//` comments up to and including their newline,
 * drop a lone '/', turn everything else into a space.  `char` reads stop at a 0xFF byte like the
 * reference's signed-char EOF test. */
static char *clean_text(const char *src, size_t n, size_t *outLen)
{
    char *o = malloc(n + 1);
    if (!o)
        return NULL;
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
        char c = src[i];
        if (c == (char)EOF)
            break;
        if ((c >= '0' && c <= '9') || c == '-' || c == '.' || c == '\n' || c == '+') {
            o[k++] = c;
        } else if (c == '/') {
            if (i + 1 < n && src[i + 1] == '/') {
                i += 2;
                while (i < n && src[i] != '\n')
                    ++i;
            }
        } else {
            o[k++] = ' ';
        }
    }
    o[k] = 0;
    *outLen = k;
    return o;
}

int rtc_parse_triangle_file(const char *path, Triangle **outTris, int *outCount)
{
    if (!path || !outTris || !outCount)
        return rtc_fail(RTC_EINVAL, "rtc_parse_triangle_file: null argument");
    *outTris = NULL;
    *outCount = 0;
    FILE *f = fopen(path, "rb");
    if (!f)
        return rtc_fail(RTC_EIO, "cannot open triangle file %s", path);
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *raw = malloc(sz > 0 ? (size_t)sz : 1);
    size_t got = sz > 0 ? fread(raw, 1, (size_t)sz, f) : 0;
    fclose(f);
    size_t clen;
    char *txt = clean_text(raw, got, &clen);
    free(raw);
    if (!txt)
        return rtc_fail(RTC_ENOMEM, "out of memory");
    /* the reference parses "<name>.parsed" (raytracing.c:78-82); we write it too, best effort */
    char parsedName[1100];
    snprintf(parsedName, sizeof parsedName, "%s.parsed", path);
    FILE *pf = fopen(parsedName, "w");
    if (pf) {
        fwrite(txt, 1, clen, pf);
        fclose(pf);
    }
    FILE *mf = fmemopen(txt, clen ? clen : 1, "r");
    if (!mf) {
        free(txt);
        return rtc_fail(RTC_ENOMEM, "fmemopen failed");
    }
    int count = 0;
    if (clen == 0 || fscanf(mf, "%i", &count) != 1 || count < 0)
        count = 0;
    Triangle *t = count ? calloc((size_t)count, sizeof(Triangle)) : NULL;
    if (count && !t) {
        fclose(mf);
        free(txt);
        return rtc_fail(RTC_ENOMEM, "out of memory");
    }
    for (int i = 0; i < count; ++i) {
        Triangle *p = &t[i];
        (void)!fscanf(mf, "%f %f %f %f %f %f %f %f %f %f %f %f %f %f", &p->posA.x, &p->posA.y, &p->posA.z, &p->posB.x,
               &p->posB.y, &p->posB.z, &p->posC.x, &p->posC.y, &p->posC.z, &p->mat.color.x, &p->mat.color.y,
               &p->mat.color.z, &p->mat.emissionStrength, &p->mat.smoothness);
        /* raytracing.c:24: counter-clockwise normal */
        p->normal = h_normalized(h_cross(h_sub(p->posB, p->posA), h_sub(p->posC, p->posA)));
    }
    fclose(mf);
    free(txt);
    *outTris = t;
    *outCount = count;
    return 0;
}

void rtc_free(void *p) { free(p); }

/* scene.h:17-19 */
static const Sphere k_default_spheres[1] = {{{0, 1, 0}, 2.5f, {{1, 1, 1}, 0, 0}}};

int rtc_default_spheres(const Sphere **outSpheres, int *outCount)
{
    if (!outSpheres || !outCount)
        return rtc_fail(RTC_EINVAL, "null argument");
    *outSpheres = k_default_spheres;
    *outCount = 1;
    return 0;
}

int rtc_scene_set_sun(Scene *scene, vec3 sunDirection)
{
    if (!scene)
        return rtc_fail(RTC_EINVAL, "null scene");
    scene->normalizedSunDirection = h_normalized(sunDirection); /* main.c:247-250 */
    return 0;
}

int rtc_default_scene(Scene *s)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "null scene");
    /* main.c:21-28 (the float conversions of the double literals happen here, as in the initialiser) */
    s->skyColorHorizon = (vec3){1, 1, 1};
    s->skyColorZenith = (vec3){(float)0.263, (float)0.969, (float)0.871};
    s->groundColor = (vec3){(float).66, (float).66, (float).66};
    s->sunFocus = 22;
    s->sunIntensity = (float).75;
    return rtc_scene_set_sun(s, (vec3){-30, -85, 100}); /* main.c:14 */
}

int rtc_camera_basis(vec3 origin, vec3 lookingAt, float fov, RtcCamera *c)
{
    if (!c)
        return rtc_fail(RTC_EINVAL, "null camera");
    /* main.c:252-255 */
    vec3 up = {0, -1, 0};
    c->origin = origin;
    c->ez = h_normalized(h_sub(lookingAt, origin));
    c->ex = h_normalized(h_cross(c->ez, up));
    c->ey = h_normalized(h_cross(c->ez, c->ex));
    c->fov = fov;
    return 0;
}

static uint8 h_float_to_uint(float f) /* moremath.c:25-30; NaN -> 0 (x86-64 cvttss2si) */
{
    if (f < 0)
        return 0;
    if (f >= 1)
        return 255;
    if (f != f)
        return 0;
    return (uint8)(f * 255.f);
}

int rtc_quantize(const float *accum, size_t pixels, Color *out)
{
    if ((!accum || !out) && pixels)
        return rtc_fail(RTC_EINVAL, "null buffer");
    for (size_t i = 0; i < pixels; ++i) {
        out[i].r = h_float_to_uint(accum[3 * i]);
        out[i].g = h_float_to_uint(accum[3 * i + 1]);
        out[i].b = h_float_to_uint(accum[3 * i + 2]);
    }
    return 0;
}

/* 24-bit BMP exactly as stbi_write_bmp writes it (stbi_image_write.h:492-500 header, :451-476 rows):
 * 14-byte file header + 40-byte BITMAPINFOHEADER, rows bottom-up, BGR, each row padded to 4 bytes. */
static void put_le(unsigned char *p, unsigned v, int n)
{
    for (int i = 0; i < n; ++i)
        p[i] = (unsigned char)(v >> (8 * i));
}

int rtc_write_bmp(const char *path, int w, int h, const Color *img)
{
    if (!path || w <= 0 || h <= 0 || !img)
        return rtc_fail(RTC_EINVAL, "rtc_write_bmp: bad argument");
    FILE *f = fopen(path, "wb");
    if (!f)
        return rtc_fail(RTC_EIO, "cannot open %s", path);
    int pad = (-w * 3) & 3;
    unsigned dataBytes = (unsigned)((w * 3 + pad) * h);
    unsigned char hd[54];
    memset(hd, 0, sizeof hd);
    hd[0] = 'B';
    hd[1] = 'M';
    put_le(hd + 2, 14 + 40 + dataBytes, 4);
    put_le(hd + 10, 14 + 40, 4);
    put_le(hd + 14, 40, 4);
    put_le(hd + 18, (unsigned)w, 4);
    put_le(hd + 22, (unsigned)h, 4);
    put_le(hd + 26, 1, 2);
    put_le(hd + 28, 24, 2);
    fwrite(hd, 1, sizeof hd, f);
    unsigned char *row = malloc((size_t)w * 3 + 4);
    if (!row) {
        fclose(f);
        return rtc_fail(RTC_ENOMEM, "out of memory");
    }
    for (int y = h - 1; y >= 0; --y) {
        const Color *src = img + (size_t)y * (size_t)w;
        for (int x = 0; x < w; ++x) {
            row[3 * x] = src[x].b;
            row[3 * x + 1] = src[x].g;
            row[3 * x + 2] = src[x].r;
        }
        memset(row + 3 * w, 0, 4);
        fwrite(row, 1, (size_t)w * 3 + (size_t)pad, f);
    }
    free(row);
    int bad = ferror(f);
    fclose(f);
    return bad ? rtc_fail(RTC_EIO, "write error on %s", path) : 0;
}
