/*
 * rtc_main.c -- command-line driver, flag-compatible with the reference's main.c:107-305.
 *
 * Same flags, defaults and exit codes as main.c (unknown flag / missing parameter -> message on stderr,
 * help on stdout, exit 0; OBJ load failure -> exit 42 as raytracing.c:109).  The render region
 * (main.c:246-304) is one rtc_render / rtc_render_multi call instead of 12 pthreads, and the framebuffer
 * lives on the heap (the reference's stack VLA, main.c:246, overflows at 4K).
 * Extra flags: --spp N (reference: compile-time 4000, scene.h:26), --gpus N, --hoist, --dump-float FILE,
 * --stats.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtc.h"

static void help(const char *prog, const char *err, const char *what, const char *after)
{
    fprintf(stderr, "%s%s%s", err, what, after);
    printf("%s [-h|--help]\n"
           "   # FILE SETTINGS\n"
           "\t[-i|--input path/to/file.obj]\n\t[-o|--output <filename>]\n"
           "   # POSITION & LOOKING-AT POSITION (TRACK)\n"
           "\t[-p|--pos <posX> <posY> <posZ>]\n\t[-t|--track <trackX> <trackY> <trackZ>]\n"
           "   # CAMERA SETTINGS\n"
           "\t[-f|--fov <fov>]\n\t[-s|--size <width> <height>]\n\t[-b|--max-bounce <maxBounce>]\n"
           "   # SCENE SETTINGS\n"
           "\t[-gc|--ground-color <R> <G> <B>]\n\t[-sch|--sky-color-horizon <R> <G> <B>]\n"
           "\t[-scz|--sky-color-zenith <R> <G> <B>]\n"
           "   # SUN SETTINGS\n"
           "\t[--sun <x> <y> <z> <focus> <intensity>]\n"
           "   # MI355X RENDERER\n"
           "\t[--spp <samples per pixel>] (default 4000)\n\t[--gpus <n>]\n\t[--hoist]\n"
           "\t[--dump-float <file>]\n\t[--stats]\n",
           prog);
    exit(0);
}

static int is(const char *a, const char *l, const char *s) { return strcmp(a, l) == 0 || (s && strcmp(a, s) == 0); }

static void need(int argc, int i, int n, const char *prog, const char *msg)
{
    if (argc - 1 < i + n)
        help(prog, msg, "", "");
}

int main(int argc, char const *argv[])
{
    char mode[256] = "default";
    char out[256] = "out.bmp";
    const char *dumpFloat = NULL;
    int width = 128, height = 128, maxBounce = 10, spp = 4000, gpus = 1, hoist = 0, stats = 0;
    vec3 origin = {-4.75f, -1.5f, -4.75f}, lookingAt = {0.9f, -1.2f, 1.f}, sunDirection = {-30, -85, 100};
    float fov = 1;
    Scene scene;
    rtc_default_scene(&scene);
    const char *p = argv[0];

    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (is(a, "--help", "-h"))
            help(p, "", "", "");
        else if (is(a, "--input", "-i")) {
            need(argc, i, 1, p, "ERROR: --input/-i takes 1 more param (string path/to/filename.obj)\n");
            snprintf(mode, sizeof mode, "%s", argv[++i]);
        } else if (is(a, "--output", "-o")) {
            need(argc, i, 1, p, "ERROR: --output/-o takes 1 more param (string outImage.bmp)\n");
            snprintf(out, sizeof out, "%s", argv[++i]);
        } else if (is(a, "--pos", "-p")) {
            need(argc, i, 3, p, "ERROR: --pos/-p takes 3 more params (float x,y,z)\n");
            origin.x = atof(argv[i + 1]), origin.y = atof(argv[i + 2]), origin.z = atof(argv[i + 3]);
            i += 3;
        } else if (is(a, "--track", "-t")) {
            need(argc, i, 3, p, "ERROR: --track/-t takes 3 more params (float x,y,z)\n");
            lookingAt.x = atof(argv[i + 1]), lookingAt.y = atof(argv[i + 2]), lookingAt.z = atof(argv[i + 3]);
            i += 3;
        } else if (is(a, "--fov", "-f")) {
            need(argc, i, 1, p, "ERROR: --fov/-i takes 1 more param (float f)\n");
            fov = atof(argv[++i]);
        } else if (is(a, "--max-bounce", "-b")) {
            need(argc, i, 1, p, "ERROR: --max-bounce/-b takes 1 more param (int f)\n");
            maxBounce = atoi(argv[++i]);
        } else if (is(a, "--size", "-s")) {
            need(argc, i, 2, p, "ERROR: --size/-s takes 2 more params (int w,h)\n");
            width = atoi(argv[i + 1]), height = atoi(argv[i + 2]);
            i += 2;
        } else if (is(a, "--ground-color", "-gc")) {
            need(argc, i, 3, p, "ERROR: --ground-color/-gc takes 3 more params (float r,g,b)\n");
            scene.groundColor = (vec3){atof(argv[i + 1]), atof(argv[i + 2]), atof(argv[i + 3])};
            i += 3;
        } else if (is(a, "--sky-color-horizon", "-sch")) {
            need(argc, i, 3, p, "ERROR: --sky-color-horizon/-sch takes 3 more params (float r,g,b)\n");
            scene.skyColorHorizon = (vec3){atof(argv[i + 1]), atof(argv[i + 2]), atof(argv[i + 3])};
            i += 3;
        } else if (is(a, "--sky-color-zenith", "-scz")) {
            need(argc, i, 3, p, "ERROR: --sky-color-zenith/-scz takes 3 more params (float r,g,b)\n");
            scene.skyColorZenith = (vec3){atof(argv[i + 1]), atof(argv[i + 2]), atof(argv[i + 3])};
            i += 3;
        } else if (is(a, "--sun", NULL)) {
            need(argc, i, 5, p, "ERROR: --sun takes 5 more params (float x,y,z,focus,intensity)\n");
            sunDirection = (vec3){atof(argv[i + 1]), atof(argv[i + 2]), atof(argv[i + 3])};
            scene.sunFocus = atof(argv[i + 4]);
            scene.sunIntensity = atof(argv[i + 5]);
            i += 5;
        } else if (is(a, "--spp", NULL)) {
            need(argc, i, 1, p, "ERROR: --spp takes 1 more param (int n)\n");
            spp = atoi(argv[++i]);
        } else if (is(a, "--gpus", NULL)) {
            need(argc, i, 1, p, "ERROR: --gpus takes 1 more param (int n)\n");
            gpus = atoi(argv[++i]);
        } else if (is(a, "--dump-float", NULL)) {
            need(argc, i, 1, p, "ERROR: --dump-float takes 1 more param (string file)\n");
            dumpFloat = argv[++i];
        } else if (is(a, "--hoist", NULL)) {
            hoist = 1;
        } else if (is(a, "--stats", NULL)) {
            stats = 1;
        } else
            help(p, "ERROR: UNKNOWN ARGUMENT \"", a, "\"\n");
    }

    printf("Starting RayTracingC in %s mode", mode);
    Triangle *tris = NULL;
    int triCount = 0, trianglesOnly = 0;
    const Sphere *spheres = NULL;
    int sphereCount = 0;
    if (strcmp(mode, "default") == 0) {
        printf("Parsing triangles...\n");
        rtc_parse_triangle_file("triangles.txt", &tris, &triCount); /* missing file: 0 triangles, as the reference */
        printf("%i triangles found\n", triCount);
        rtc_default_spheres(&spheres, &sphereCount);
    } else {
        trianglesOnly = 1;
        printf("Loading obj...\n");
        if (rtc_load_obj(mode, &tris, &triCount) != 0) {
            fprintf(stderr, "%s", rtc_last_error());
            return 42;
        }
    }
    rtc_scene_set_sun(&scene, sunDirection);
    RtcCamera cam;
    rtc_camera_basis(origin, lookingAt, fov, &cam);
    if (width <= 0 || height <= 0) {
        fprintf(stderr, "invalid size %dx%d\n", width, height);
        return 1;
    }
    size_t px = (size_t)width * (size_t)height;
    Color *image = calloc(px, sizeof(Color));
    float *accum = dumpFloat ? calloc(px * 3, sizeof(float)) : NULL;
    RtcRenderDesc d = {width, height, spp, maxBounce, trianglesOnly, 0, 1, hoist ? RTC_F_HOIST_PRIMARY : 0};
    RtcStats st;
    memset(&st, 0, sizeof st);
    printf("Starting RENDERING...\n");
    int rc = gpus > 1 ? rtc_render_multi(tris, triCount, spheres, sphereCount, &scene, &cam, &d, gpus, image, accum, &st)
                      : rtc_render(tris, triCount, spheres, sphereCount, &scene, &cam, &d, -1, image, accum, &st);
    if (rc != 0) {
        fprintf(stderr, "render failed (%d): %s\n", rc, rtc_last_error());
        return 2;
    }
    if (stats)
        printf("frame %.3f ms (render %.3f ms), %.1f Mrays/s, %llu segments\n", st.frameMs, st.renderMs,
               st.frameMs > 0 ? (double)st.samples / (st.frameMs * 1e3) : 0.0, st.segments);
    if (rtc_write_bmp(out, width, height, image) != 0)
        fprintf(stderr, "%s\n", rtc_last_error());
    if (dumpFloat) {
        FILE *f = fopen(dumpFloat, "wb");
        if (f) {
            fwrite(&width, 4, 1, f);
            fwrite(&height, 4, 1, f);
            fwrite(accum, sizeof(float), px * 3, f);
            fclose(f);
        }
    }
    free(image);
    free(accum);
    rtc_free(tris);
    return 0;
}
