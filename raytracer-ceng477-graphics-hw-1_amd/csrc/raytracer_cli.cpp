// Drop-in replacement for the reference executable (raytracer.cpp:487-525):
//
//   ./raytracer scene.xml            -> writes every camera's ImageName into CWD
//
// Same stdout lines as the reference ("Planted trees in ...", the SSAA notice,
// "Rendering <name> with ...", "Rendered in ...", "Total: ...") and the same
// default SSAA factor 2 (raytracer.cpp:26-28).  Extra flags:
//   --aa F           SSAA factor (1 disables, as DO_SSAA_ANTI_ALIASING false)
//   --max-depth D    override MaxRecursionDepth
//   --device N       HIP device ordinal
//   --gpus N         render every frame on GPUs 0..N-1 (row stripes + one RCCL gather, rt_set_devices)
//   --no-write       skip write_ppm (timing)
//   --timing         a JSON line on stderr: steady-clock stamps (ms) of main's phases and the scene-build split
// The process ends with _exit once every image is written and stdout flushed: the HIP runtime's teardown at a
// normal exit costs tens of ms and frees nothing the OS does not (RT_CLI_EXIT=normal: a normal exit).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt/rt.h"

namespace {

double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int die(const char* what) {
    std::fprintf(stderr, "%s: %s\n", what, rt_last_error());
    return 1;
}

}  // namespace

double stamp() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const double t_main = stamp();
    // several cameras render as concurrent frame batches, one stream each: give HIP enough hardware
    // queues that they do not share (read at the runtime's first use).  RT_HW_QUEUES overrides; a
    // GPU_MAX_HW_QUEUES the user already set is kept; otherwise 8.
    if (const char* q = std::getenv("RT_HW_QUEUES")) setenv("GPU_MAX_HW_QUEUES", q, 1);
    else setenv("GPU_MAX_HW_QUEUES", "8", 0);
    const char* scene_path = nullptr;
    int aa = 2, max_depth = -1000, device = 0, gpus = 0;   // device 0 unless --device: an explicit device lets
                                                          // the library start HIP while the XML is read
    bool write = true, timing = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--aa") && i + 1 < argc) aa = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--max-depth") && i + 1 < argc) max_depth = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--no-write")) write = false;
        else if (!std::strcmp(argv[i], "--timing")) timing = true;
        else if (argv[i][0] != '-' && !scene_path) scene_path = argv[i];
        else {
            std::fprintf(stderr, "usage: %s scene.xml [--aa F] [--max-depth D] [--device N] [--gpus N] [--no-write] [--timing]\n", argv[0]);
            return 2;
        }
    }
    if (!scene_path || aa < 1) {
        std::fprintf(stderr, "usage: %s scene.xml [--aa F] [--max-depth D] [--device N] [--gpus N] [--no-write]\n", argv[0]);
        return 2;
    }

    if (gpus > 0 && rt_set_devices(gpus) != RT_OK) return die("gpus");
    const auto begin1 = std::chrono::steady_clock::now();
    rt_options opts{device, 0, 0};
    rt_scene* scene = nullptr;
    if (rt_scene_load_xml(scene_path, &opts, &scene) != RT_OK) return die("load");
    if (max_depth != -1000 && rt_scene_set_max_depth(scene, max_depth) != RT_OK) return die("max-depth");
    const double planted = seconds_since(begin1);
    const double t_load = stamp();
    std::printf("Planted trees in %.3f seconds.\n", planted);
    if (aa > 1) std::printf("Super Sampling Anti aliasing is enabled. (%d*%dx)\n", aa, aa);

    const auto begin2 = std::chrono::steady_clock::now();
    // all cameras in one batched call (frames run concurrently on the GPU), then write_ppm each
    const int ncam = rt_scene_num_cameras(scene);
    std::vector<rt_camera> cams(ncam);
    std::vector<std::string> names(ncam);
    std::vector<std::vector<uint8_t>> imgs(ncam);
    std::vector<uint8_t*> outs(ncam);
    for (int c = 0; c < ncam; ++c) {
        char name[1024];
        if (rt_scene_get_camera(scene, c, &cams[c], name, sizeof name) != RT_OK) return die("camera");
        names[c] = name;
        std::printf("Rendering %s on %d GPU(s) (SSAA %dx%d)...\n", name, rt_scene_num_devices(scene), aa, aa);
        imgs[c].resize((size_t)cams[c].image_width * cams[c].image_height * 3);
        outs[c] = imgs[c].data();
    }
    std::fflush(stdout);
    if (ncam > 0 && rt_render_cameras(scene, cams.data(), ncam, aa, outs.data(), nullptr) != RT_OK) return die("render");
    const double t_render = stamp();
    for (int c = 0; c < ncam && write; ++c)
        if (rt_write_ppm(names[c].c_str(), imgs[c].data(), cams[c].image_width, cams[c].image_height) != RT_OK)
            return die("write_ppm");
    const double t_write = stamp();
    const double rendered = seconds_since(begin2);
    std::printf("Rendered in %.3f seconds.\n", rendered);
    std::printf("Total: %.3f seconds.\n", rendered + planted);
    std::fflush(stdout);
    if (timing) {
        rt_bvh_info bi{};
        rt_scene_bvh_info(scene, &bi);
        std::fprintf(stderr,
                     "{\"cli\": {\"main\": %.3f, \"loaded\": %.3f, \"rendered\": %.3f, \"written\": %.3f, "
                     "\"xml_ms\": %.3f, \"prep_ms\": %.3f, \"ref_tree_ms\": %.3f, \"flat_ms\": %.3f, \"refwide_ms\": %.3f, "
                     "\"stree_ms\": %.3f, \"upload_ms\": %.3f}}\n",
                     t_main, t_load, t_render, t_write, bi.xml_ms, bi.prep_ms, bi.ref_ms, bi.flat_ms, bi.refwide_ms,
                     bi.stree_ms, bi.upload_ms);
        std::fflush(stderr);
    }
    const char* ex = std::getenv("RT_CLI_EXIT");
    if (!ex || std::strcmp(ex, "normal")) std::_Exit(0);   // (every file is closed by rt_write_ppm)
    rt_scene_destroy(scene);
    return 0;
}
