/* ORACLE / TEST INFRASTRUCTURE ONLY: command-line driver for rt_oracle.c.
 *   rt_oracle_cli scene.xml [--aa F] [--threads T] [--camera i] [--out-dir D] [--raw-dir D]
 * Prints one JSON line per camera with the work counters. */
#define _GNU_SOURCE
#include "rt_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }

int main(int argc, char** argv) {
    const char* scene = NULL; const char* out_dir = NULL; const char* raw_dir = NULL;
    int aa = 1, threads = 8, camera = -1;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--aa") && i + 1 < argc) aa = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--camera") && i + 1 < argc) camera = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--out-dir") && i + 1 < argc) out_dir = argv[++i];
        else if (!strcmp(argv[i], "--raw-dir") && i + 1 < argc) raw_dir = argv[++i];
        else scene = argv[i];
    }
    if (!scene) { fprintf(stderr, "usage: rt_oracle_cli scene.xml [--aa F] [--threads T]\n"); return 2; }
    char err[256];
    double t0 = now_s();
    ro_scene* s = ro_load(scene, err, sizeof err);
    if (!s) { fprintf(stderr, "%s\n", err); return 1; }
    double t_load = now_s() - t0;
    int nodes, leaves, ml, nt, ns; ro_bvh_info(s, &nodes, &leaves, &ml, &nt, &ns);
    printf("{\"event\": \"load\", \"seconds\": %.6f, \"nodes\": %d, \"leaves\": %d, \"max_leaf\": %d, \"tris\": %d, \"spheres\": %d}\n",
           t_load, nodes, leaves, ml, nt, ns);
    for (int c = 0; c < ro_num_cameras(s); ++c) {
        if (camera >= 0 && c != camera) continue;
        int W, H; char name[256]; ro_camera_info(s, c, &W, &H, name, sizeof name);
        unsigned char* img = (unsigned char*)malloc((size_t)W * H * 3);
        ro_counters k;
        double t1 = now_s();
        ro_render(s, c, aa, threads, 0, H, -1000, img, &k);
        double dt = now_s() - t1;
        printf("{\"event\": \"render\", \"camera\": %d, \"image\": \"%s\", \"aa\": %d, \"seconds\": %.6f, "
               "\"primary\": %llu, \"shadow\": %llu, \"reflection\": %llu, \"node_visits\": %llu, "
               "\"tri_tests\": %llu, \"sphere_tests\": %llu}\n",
               c, name, aa, dt, (unsigned long long)k.primary_rays, (unsigned long long)k.shadow_rays,
               (unsigned long long)k.reflection_rays, (unsigned long long)k.node_visits,
               (unsigned long long)k.tri_tests, (unsigned long long)k.sphere_tests);
        char path[1024];
        if (out_dir) { snprintf(path, sizeof path, "%s/%s", out_dir, name); ro_write_ppm(path, img, W, H); }
        if (raw_dir) {
            snprintf(path, sizeof path, "%s/%s.rgb", raw_dir, name);
            FILE* f = fopen(path, "wb"); if (f) { fwrite(img, 1, (size_t)W * H * 3, f); fclose(f); }
        }
        free(img);
    }
    ro_free(s);
    return 0;
}
