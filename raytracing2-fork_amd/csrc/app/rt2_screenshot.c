/*
 * rt2_screenshot — the offline render of the reference (screenshot(),
 * RayTracing/src/rayTracing.cpp:124-283, driven from main() :1210-1443) as a
 * plain C program over the rt2 C-ABI: load the model folder, append the five
 * materials main() appends (:1268-1283), build the chosen box, build the BVH
 * (fixes the triangle order), fill the uniforms, render on the GPU, average,
 * flip, write the PNG.
 *
 *   rt2_screenshot [--model DIR] [--box cornell|mirror|sidelit|sky|classic|diverse|none]
 *                  [--width W] [--height H] [--rays R] [--frames F] [--bounces B]
 *                  [--out PATH] [--float-mean] [--device D] [--traversal brute|bvh]
 *                  [--nranks N --rank R --id-file PATH [--tile-rows T]]
 *
 * Default output is the reference's 8-bit path (per-frame unorm8, float sum,
 * truncating average: rayTracing.cpp:217-250); --float-mean writes the
 * mean of the float frames quantised once instead.
 *
 * Multi-GPU: start one process per GPU with the same
 * arguments plus --nranks N --rank R (and --device, default R).  Rank 0 writes
 * the RCCL communicator id to --id-file, the others read it; every rank
 * renders the row tiles of rt2_shard {T, R, N}, one RCCL gather brings the
 * slabs to rank 0, which writes the PNG (identical to a one-GPU run).
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../../include/rt2.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int die(const char* what) {
    fprintf(stderr, "rt2_screenshot: %s: %s\n", what, rt2_last_error());
    return 1;
}

/* The communicator id travels through a file: rank 0 writes it under a
 * temporary name and renames it (atomic), the other ranks poll for it. */
static int exchange_id(const char* path, int rank, uint8_t* id) {
    if (rank == 0) {
        if (rt2_comm_unique_id(id)) return die("rt2_comm_unique_id");
        char tmp[4096];
        snprintf(tmp, sizeof tmp, "%s.tmp%d", path, (int)getpid());
        FILE* f = fopen(tmp, "wb");
        if (!f || fwrite(id, 1, RT2_COMM_ID_BYTES, f) != RT2_COMM_ID_BYTES || fclose(f) != 0 || rename(tmp, path)) {
            fprintf(stderr, "rt2_screenshot: cannot write %s\n", path);
            return 1;
        }
        return 0;
    }
    for (int tries = 0; tries < 6000; tries++) {  /* 60 s */
        FILE* f = fopen(path, "rb");
        if (f) {
            size_t got = fread(id, 1, RT2_COMM_ID_BYTES, f);
            fclose(f);
            if (got == RT2_COMM_ID_BYTES) return 0;
        }
        struct timespec ts = {0, 10000000};
        nanosleep(&ts, NULL);
    }
    fprintf(stderr, "rt2_screenshot: no communicator id in %s after 60 s\n", path);
    return 1;
}

int main(int argc, char** argv) {
    const char* model = NULL;
    const char* box = "cornell";
    const char* out = "test.png";
    const char* id_file = NULL;
    int W = 1000, H = 1000, R = 64, F = 10, B = 20, device = -1, float_mean = 0;
    int nranks = 0, rank = 0, tile_rows = 1, bvh = 0;
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "--model") && v) model = argv[++i];
        else if (!strcmp(a, "--box") && v) box = argv[++i];
        else if (!strcmp(a, "--out") && v) out = argv[++i];
        else if (!strcmp(a, "--width") && v) W = atoi(argv[++i]);
        else if (!strcmp(a, "--height") && v) H = atoi(argv[++i]);
        else if (!strcmp(a, "--rays") && v) R = atoi(argv[++i]);
        else if (!strcmp(a, "--frames") && v) F = atoi(argv[++i]);
        else if (!strcmp(a, "--bounces") && v) B = atoi(argv[++i]);
        else if (!strcmp(a, "--device") && v) device = atoi(argv[++i]);
        else if (!strcmp(a, "--nranks") && v) nranks = atoi(argv[++i]);
        else if (!strcmp(a, "--rank") && v) rank = atoi(argv[++i]);
        else if (!strcmp(a, "--tile-rows") && v) tile_rows = atoi(argv[++i]);
        else if (!strcmp(a, "--id-file") && v) id_file = argv[++i];
        else if (!strcmp(a, "--traversal") && v) bvh = !strcmp(argv[++i], "bvh");
        else if (!strcmp(a, "--float-mean")) float_mean = 1;
        else {
            fprintf(stderr, "unknown argument %s\n", a);
            return 2;
        }
    }

    if (nranks > 0 && (!id_file || rank < 0 || rank >= nranks || tile_rows < 1)) {
        fprintf(stderr, "rank mode needs --id-file, 0 <= --rank < --nranks and --tile-rows >= 1\n");
        return 2;
    }
    if (device < 0) device = nranks > 0 ? rank : 0;

    rt2_scene_data* sd = rt2_sd_create();
    if (!sd) return die("rt2_sd_create");
    if (model && rt2_sd_load_obj_folder(sd, model)) return die("load model");
    if (!model) {  /* the no-OBJ path (config A): a default material at index 0 */
        rt2_material d;
        rt2_material_default(&d);
        rt2_sd_add_material(sd, &d);
    }
    rt2_material m;
    rt2_material_default(&m); rt2_material_make_diffuse(&m, 1.0f, 0.0f, 0.0f);
    int red = rt2_sd_add_material(sd, &m);
    rt2_material_default(&m); rt2_material_make_diffuse(&m, 0.0f, 1.0f, 0.0f);
    int green = rt2_sd_add_material(sd, &m);
    rt2_material_default(&m); rt2_material_make_diffuse(&m, 1.0f, 1.0f, 1.0f);
    int wall = rt2_sd_add_material(sd, &m);
    rt2_material_default(&m); rt2_material_make_light(&m, 1.0f, 1.0f, 1.0f, 15.0f);
    int light = rt2_sd_add_material(sd, &m);
    rt2_material_default(&m); rt2_material_make_specular(&m, 1, 1, 1, 1, 1, 1, 1.0f, 1.0f);
    int mirror = rt2_sd_add_material(sd, &m);

    int rc = 0;
    if (!strcmp(box, "cornell")) rc = rt2_sd_add_cornell_box(sd, 0.17f, 0.3f, light, 1);
    else if (!strcmp(box, "mirror")) rc = rt2_sd_add_mirror_cornell_box(sd, 0.17f, 0.3f, light, mirror);
    else if (!strcmp(box, "sidelit")) rc = rt2_sd_add_side_lit_cornell_box(sd, 0.17f, 0.3f, light, wall, 1);
    else if (!strcmp(box, "sky")) rc = rt2_sd_add_sky_light_plane(sd, light);
    else if (!strcmp(box, "classic")) rc = rt2_sd_create_classic_cornell_box(sd, 10.0f, red, green, wall, light);
    else if (!strcmp(box, "diverse")) {
        rt2_material_default(&m); rt2_material_make_glass(&m, 1, 1, 1, 1.5f);
        int glass = rt2_sd_add_material(sd, &m);
        rt2_material_default(&m); rt2_material_make_checker(&m, 10.0f);
        int checker = rt2_sd_add_material(sd, &m);
        rt2_material_default(&m); rt2_material_make_specular(&m, 0.8f, 0.8f, 0.8f, 1, 1, 1, 0.9f, 0.5f);
        int metal = rt2_sd_add_material(sd, &m);
        rc = rt2_sd_create_diverse_cornell_box(sd, 10.0f, red, green, wall, light, glass, mirror, checker, metal);
    } else if (strcmp(box, "none")) {
        fprintf(stderr, "unknown --box %s\n", box);
        return 2;
    }
    if (rc) return die("scene builder");
    if (rt2_sd_build_bvh(sd)) return die("BVH");
    printf("%d triangles, %d materials, %d BVH nodes\n", rt2_sd_num_triangles(sd), rt2_sd_num_materials(sd),
           rt2_sd_num_nodes(sd));

    rt2_uniforms u;
    rt2_uniforms_offline(&u, W, H, B, R, rt2_sd_num_triangles(sd), 0);
    rt2_comm* comm = NULL;
    if (nranks > 0) {  /* joins the other ranks (blocks until all have) */
        uint8_t id[RT2_COMM_ID_BYTES];
        if (exchange_id(id_file, rank, id)) return 1;
        if (rt2_comm_init(id, nranks, rank, device, &comm)) return die("rt2_comm_init");
    }
    rt2_scene* scene = NULL;
    double t0 = now_s();
    if (rt2_scene_create(rt2_sd_triangles(sd), rt2_sd_num_triangles(sd), rt2_sd_materials(sd), rt2_sd_num_materials(sd),
                         rt2_sd_nodes(sd), rt2_sd_num_nodes(sd), device, &scene))
        return die("rt2_scene_create");
    if (bvh && rt2_scene_set_traversal(scene, RT2_TRAVERSAL_BVH)) return die("traversal");
    double t1 = now_s();
    size_t n = (size_t)W * (size_t)H;
    float* rgba = (float*)malloc(n * 16);
    unsigned char* rgb8 = (unsigned char*)malloc(n * 3);
    if (!rgba || !rgb8) return die("malloc");
    if (nranks > 0) {
        rt2_shard sh = {tile_rows, rank, nranks};
        if (rt2_render_host_gather(scene, &u, 0, (uint32_t)F, sh, comm, 0, rgba, rgb8)) return die("render");
    } else {
        rt2_shard all = {1, 0, 1};
        if (rt2_render_host(scene, &u, 0, (uint32_t)F, all, rgba, rgb8)) return die("render");
    }
    double t2 = now_s();
    rt2_stats st;
    rt2_scene_stats(scene, &st, 1);
    printf("upload %.3f s, render %.3f s, %.2f Msamples/s, %llu segments\n", t1 - t0, t2 - t1,
           (double)st.samples / (t2 - t1) * 1e-6, (unsigned long long)st.segments);
    if (comm) rt2_comm_destroy(comm);
    if (rank != 0) {  /* the image lives on rank 0 */
        free(rgba);
        free(rgb8);
        rt2_scene_destroy(scene);
        rt2_sd_destroy(sd);
        return 0;
    }

    if (float_mean)
        for (size_t i = 0; i < n; i++)
            for (int c = 0; c < 3; c++) {
                float v = rgba[4 * i + c] * 255.0f + 0.5f;
                /* NaN -> 0 (a NaN reaching the unsigned char conversion is undefined) */
                rgb8[3 * i + c] = (unsigned char)(v > 255.0f ? 255.0f : (v >= 0.0f ? v : 0.0f));
            }
    /* vertical flip, rayTracing.cpp:253-259 */
    for (int y = 0; y < H / 2; y++)
        for (int x = 0; x < W * 3; x++) {
            size_t a = (size_t)y * W * 3 + x, b = (size_t)(H - 1 - y) * W * 3 + x;
            unsigned char t = rgb8[a];
            rgb8[a] = rgb8[b];
            rgb8[b] = t;
        }
    if (rt2_write_png(out, W, H, 3, rgb8, W * 3)) return die("write png");
    printf("Screenshot saved to: %s\n", out);
    free(rgba);
    free(rgb8);
    rt2_scene_destroy(scene);
    rt2_sd_destroy(sd);
    return 0;
}
