// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Harness around the *unmodified* reference renderer.  It is compiled by
// oracle/Makefile directly from the sources where they lie
// (/root/reference/raytracer.cpp, parser.cpp, ppm.cpp, tinyxml2.cpp); nothing
// from the reference is copied into this repository.  Output goes to
// oracle/_ref/ (git-ignored).
//
// Why a harness and not the stock binary: the stock `main`
// (raytracer.cpp:487-525) hard-codes SSAA factor 2 (raytracer.cpp:26-28),
// spawns hardware_concurrency() threads (raytracer.cpp:367) and always writes
// every camera.  To produce parity goldens for AA 1/2/4, derived configs and
// per-pixel primary hit-t dumps we drive the reference's own public classes:
//   RayTracer ctor (raytracer.cpp:335-350)          -> BVH build
//   RayTracer::renderWithMultipleThreads (:352-360) -> the per-pixel hot loop
//   ImageProcessor::downSample (:459-484)           -> SSAA box filter
//   write_ppm (ppm.cpp:4-39)                        -> P3 output
//   EyeRayGenerator::generate + Ray::getFirstIntersection (:319-324, :177-225)
//                                                   -> primary hit-t dump
#define main reference_main
#include "raytracer.cpp"
#undef main

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Args {
    const char* scene = nullptr;
    int aa = 1;
    int threads = 0;
    int camera = -1;           // -1 = all cameras
    int reps = 1;
    int max_depth = -1000;     // override of MaxRecursionDepth (parser.cpp:48-57)
    int width = 0, height = 0; // override of ImageResolution
    bool has_near = false;
    float near_plane[4] = {0, 0, 0, 0};
    const char* out_dir = nullptr;  // write <ImageName> (P3) here
    const char* raw_dir = nullptr;  // write <ImageName>.rgb (raw u8) here
    const char* dump_t = nullptr;   // primary-ray {t, material, exists} dump (internal res)
    int rows = -1;                  // render only the first `rows` output rows (bounded CPU sample)
};

void usage() {
    fprintf(stderr,
            "ref_harness scene.xml [--aa F] [--threads T] [--camera i] [--reps N]\n"
            "            [--max-depth D] [--res W H] [--near l r b t]\n"
            "            [--out-dir D] [--raw-dir D] [--dump-t file] [--rows R]\n");
    exit(2);
}

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string s = argv[i];
        auto need = [&](int n) { if (i + n >= argc) usage(); };
        if (s == "--aa") { need(1); a.aa = atoi(argv[++i]); }
        else if (s == "--threads") { need(1); a.threads = atoi(argv[++i]); }
        else if (s == "--camera") { need(1); a.camera = atoi(argv[++i]); }
        else if (s == "--reps") { need(1); a.reps = atoi(argv[++i]); }
        else if (s == "--max-depth") { need(1); a.max_depth = atoi(argv[++i]); }
        else if (s == "--res") { need(2); a.width = atoi(argv[++i]); a.height = atoi(argv[++i]); }
        else if (s == "--near") {
            need(4); a.has_near = true;
            for (int k = 0; k < 4; ++k) a.near_plane[k] = strtof(argv[++i], nullptr);
        }
        else if (s == "--out-dir") { need(1); a.out_dir = argv[++i]; }
        else if (s == "--raw-dir") { need(1); a.raw_dir = argv[++i]; }
        else if (s == "--dump-t") { need(1); a.dump_t = argv[++i]; }
        else if (s == "--rows") { need(1); a.rows = atoi(argv[++i]); }
        else if (s[0] != '-' && !a.scene) a.scene = argv[i];
        else usage();
    }
    if (!a.scene || a.aa < 1) usage();
    return a;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Same fork/join as RayTracer::render (raytracer.cpp:362-383) but with an
// explicit thread count, so the CPU baseline uses exactly the cores we state.
Image render_threads(RayTracer& rt, Camera& cam, int T, int rows_limit) {
    int full_h = cam.image_height;
    if (rows_limit >= 0) cam.image_height = std::min(full_h, rows_limit);
    auto image = new Pixel[(size_t)cam.image_width * full_h];
    memset(image, 0, (size_t)cam.image_width * full_h * 3);
    rt.currentCamera = &cam;
    rt.currentImage = image;
    rt.eyeRayGenerator.init(rt.currentCamera);
    // eyeRayGenerator.init used the (possibly truncated) height for svMultiplier;
    // restore the full-frame pitch so the bounded sample is a true sub-frame.
    if (rows_limit >= 0) {
        Camera full = cam;
        full.image_height = full_h;
        rt.eyeRayGenerator.init(&full);
    }
    std::vector<std::thread> threads;
    for (int i = 0; i < T; ++i)
        threads.emplace_back(&RayTracer::renderWithMultipleThreads, &rt, i, T);
    for (auto& t : threads) t.join();
    cam.image_height = full_h;
    return image;
}

}  // namespace

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    parser::Scene scene;
    const double tl0 = now_s();
    scene.loadFromXml(a.scene);
    printf("{\"event\": \"load\", \"seconds\": %.6f}\n", now_s() - tl0);
    if (a.max_depth != -1000) scene.max_recursion_depth = a.max_depth;
    for (auto& c : scene.cameras) {
        if (a.width > 0) { c.image_width = a.width; c.image_height = a.height; }
        if (a.has_near) {
            c.near_plane.x = a.near_plane[0]; c.near_plane.y = a.near_plane[1];
            c.near_plane.z = a.near_plane[2]; c.near_plane.w = a.near_plane[3];
        }
    }
    int T = a.threads > 0 ? a.threads : (int)std::max(1u, std::thread::hardware_concurrency());

    double t0 = now_s();
    RayTracer rayTracer(scene);
    double t_build = now_s() - t0;
    printf("{\"event\": \"bvh\", \"seconds\": %.6f, \"nodes\": %zu}\n", t_build, rayTracer.tree.nodes.size());

    for (size_t ci = 0; ci < scene.cameras.size(); ++ci) {
        if (a.camera >= 0 && (int)ci != a.camera) continue;
        Camera camera = scene.cameras[ci];
        camera.image_width *= a.aa;
        camera.image_height *= a.aa;
        int rows_internal = a.rows >= 0 ? a.rows * a.aa : -1;
        std::vector<double> times;
        Image image = nullptr;
        for (int r = 0; r < a.reps; ++r) {
            if (image) delete[] image;
            double s = now_s();
            image = render_threads(rayTracer, camera, T, rows_internal);
            times.push_back(now_s() - s);
        }
        std::sort(times.begin(), times.end());
        int ow = camera.image_width / a.aa, oh = camera.image_height / a.aa;
        if (a.aa > 1) {
            Image ds = ImageProcessor::downSample(image, camera.image_width, camera.image_height, a.aa);
            delete[] image;
            image = ds;
        }
        printf("{\"event\": \"render\", \"camera\": %zu, \"image\": \"%s\", \"width\": %d, \"height\": %d, "
               "\"aa\": %d, \"threads\": %d, \"rows\": %d, \"median_s\": %.6f, \"min_s\": %.6f}\n",
               ci, camera.image_name.c_str(), ow, oh, a.aa, T, a.rows, times[times.size() / 2], times[0]);
        if (a.out_dir) {
            std::string p = std::string(a.out_dir) + "/" + camera.image_name;
            write_ppm(p.c_str(), (unsigned char*)image, ow, oh);
        }
        if (a.raw_dir) {
            std::string p = std::string(a.raw_dir) + "/" + camera.image_name + ".rgb";
            FILE* f = fopen(p.c_str(), "wb");
            if (!f) { perror(p.c_str()); return 1; }
            fwrite(image, 1, (size_t)ow * oh * 3, f);
            fclose(f);
        }
        if (a.dump_t) {
            // Primary rays at internal resolution: record {t, material_id, exists}
            // exactly as Ray::getFirstIntersection returns them (raytracer.cpp:177-225).
            rayTracer.eyeRayGenerator.init(&camera);
            int W = camera.image_width, H = camera.image_height;
            std::vector<float> tt((size_t)W * H);
            std::vector<int> mm((size_t)W * H);
            for (int row = 0; row < H; ++row)
                for (int col = 0; col < W; ++col) {
                    Ray ray = rayTracer.eyeRayGenerator.generate(row, col);
                    Intersection in = ray.getFirstIntersection(rayTracer.scene, rayTracer.tree);
                    tt[(size_t)row * W + col] = in.tSmall;
                    mm[(size_t)row * W + col] = in.exists ? in.material_id : 0;
                }
            FILE* f = fopen(a.dump_t, "wb");
            if (!f) { perror(a.dump_t); return 1; }
            fwrite(tt.data(), 4, tt.size(), f);
            fwrite(mm.data(), 4, mm.size(), f);
            fclose(f);
        }
        delete[] image;
    }
    return 0;
}
