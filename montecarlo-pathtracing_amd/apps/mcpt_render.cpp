// mcpt_render — headless entry point of the MI355X path tracer (the montecarlo.cpp main,
// MontecarloGPU/montecarlo.cpp:797-803, without the GL window).
//
// Builds one of the 8 reference scenes (keys Q..I = 1..8), accumulates passes with the
// reference's uniform ABI (numero_pass, date, NB_BOUNCES, refract_ind, shader variant),
// progressively in chunks like the "lock" mode (optionally writing a checkpoint after each
// chunk, and resuming from one), then writes the averaged image (fs_frag,
// montecarlo.cpp:59-70) as PFM (float) and/or PNG (8-bit framebuffer view).  Prints one JSON
// line with the timing.  Host C++ over the C ABI (include/mcpt.hpp); no CPU fallback.
//
// Several GPUs (--devices 0,1,...,7): one context and one host thread per device, each
// rendering its rows of the balanced row partition (mcpt_balanced_rows) for all
// passes; the shards' rows are then copied device to device into a full frame on the first
// device (mcpt_gather_rows: peer copies over xGMI — no collective on the data path).  The
// bits equal the one-GPU render's.  A device may be listed more than once (shards sharing a
// GPU: the 1-GPU rehearsal of the N-GPU path).
//
//   mcpt_render --scene 6 --width 1920 --height 1080 --spp 256 --bounces 8 --out s6.png
//   mcpt_render --scene 8 --width 1920 --height 1080 --spp 512 --bounces 12 --devices 0,1,2,3,4,5,6,7
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mcpt.hpp"

namespace {

struct Args {
  int scene = 6, width = 1280, height = 1000, spp = 16, bounces = 3, first_pass = 1, chunk = 64;
  int device = 0, subsampling = 0, variant = MCPT_MONTECARLO, traversal = MCPT_TRAVERSAL_AUTO;
  float ior = 1.0f, light = 1.2f, date = 0.0f;
  std::string png, pfm;
  std::string checkpoint, resume;   // --checkpoint FILE (after every chunk), --resume FILE
  std::vector<int> devices;   // --devices: one shard per entry
};

bool parse_list(const char* v, std::vector<int>& out) {
  out.clear();
  for (const char* p = v; *p;) {
    char* end = nullptr;
    const long d = std::strtol(p, &end, 10);
    if (end == p || d < 0 || d > 1024) return false;
    if (*end && *end != ',') return false;
    out.push_back((int)d);
    p = (*end == ',') ? end + 1 : end;
  }
  return !out.empty();
}

void usage() {
  std::fprintf(stderr,
               "usage: mcpt_render [--scene 1..8] [--width W] [--height H] [--subsampling k]\n"
               "                   [--spp S] [--first-pass P] [--chunk C] [--bounces B] [--ior R]\n"
               "                   [--light L] [--date T] [--variant montecarlo|mat|mat_tr]\n"
               "                   [--traversal auto|lane|wave|stream] [--device D | --devices D0,D1,...]\n"
               "                   [--out img.png] [--pfm img.pfm]\n"
               "                   [--checkpoint state.ckpt] [--resume state.ckpt]   (one device)\n");
}

bool parse(int argc, char** argv, Args& a) {
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    if (k == "-h" || k == "--help") return false;
    if (i + 1 >= argc) return false;
    const char* v = argv[++i];
    if (k == "--scene") a.scene = std::atoi(v);
    else if (k == "--width") a.width = std::atoi(v);
    else if (k == "--height") a.height = std::atoi(v);
    else if (k == "--subsampling") a.subsampling = std::atoi(v);
    else if (k == "--spp") a.spp = std::atoi(v);
    else if (k == "--first-pass") a.first_pass = std::atoi(v);
    else if (k == "--chunk") a.chunk = std::atoi(v);
    else if (k == "--bounces") a.bounces = std::atoi(v);
    else if (k == "--ior") a.ior = (float)std::atof(v);
    else if (k == "--light") a.light = (float)std::atof(v);
    else if (k == "--date") a.date = (float)std::atof(v);
    else if (k == "--device") a.device = std::atoi(v);
    else if (k == "--devices") {
      if (!parse_list(v, a.devices)) return false;
    }
    else if (k == "--out") a.png = v;
    else if (k == "--pfm") a.pfm = v;
    else if (k == "--checkpoint") a.checkpoint = v;
    else if (k == "--resume") a.resume = v;
    else if (k == "--variant") {
      const std::string s = v;
      a.variant = s == "mat" ? MCPT_MAT : (s == "mat_tr" ? MCPT_MAT_TR : MCPT_MONTECARLO);
      if (s != "mat" && s != "mat_tr" && s != "montecarlo") return false;
    } else if (k == "--traversal") {
      const std::string s = v;
      a.traversal = s == "lane"     ? MCPT_TRAVERSAL_LANE
                    : s == "wave"   ? MCPT_TRAVERSAL_WAVE
                    : s == "stream" ? MCPT_TRAVERSAL_STREAM
                                    : MCPT_TRAVERSAL_AUTO;
    } else {
      return false;
    }
  }
  if (!a.devices.empty() && (!a.checkpoint.empty() || !a.resume.empty())) return false;   // one device only
  return a.width > 0 && a.height > 0 && a.spp >= 0 && a.chunk > 0 && a.subsampling >= 0 && a.subsampling < 16;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse(argc, argv, a)) {
    usage();
    return 2;
  }
  try {
    mcpt::BVH_GPU_Scene scene;
    scene.build_reference(a.scene, a.light);
    // sub-sampling renders the FBO at (W>>k) x (H>>k) with the window's aspect (montecarlo.cpp:616-626)
    const int W = a.width >> a.subsampling, H = a.height >> a.subsampling;
    if (W <= 0 || H <= 0) throw std::runtime_error("sub-sampled framebuffer is empty");
    const mcpt::Camera cam = mcpt::Camera::canonical(a.width, a.height);

    double kernel_ms = 0.0, wall_ms = 0.0, gather_ms = 0.0;
    std::vector<float> img;
    std::string shard_json;
    if (a.devices.empty()) {
      mcpt::Renderer r(a.device);
      r.set_traversal(a.traversal);
      r.upload(scene);
      r.set_target(W, H);
      // checkpoint / resume: --spp counts the whole render's passes (first_pass .. first_pass +
      // spp - 1); a resumed run continues at the checkpoint's next pass with its sums loaded,
      // and the tag makes a resume with other render parameters fail
      char tag[256];
      // (the chunk too: a call that splits a 32-pass accumulation chunk adds its own partial sum,
      // so the resumed bits equal the uninterrupted run's only with the same call boundaries)
      std::snprintf(tag, sizeof(tag),
                    "scene=%d W=%d H=%d bounces=%d ior=%a light=%a date=%a variant=%d first=%d chunk=%d", a.scene, W,
                    H, a.bounces, a.ior, a.light, a.date, a.variant, a.first_pass, a.chunk);
      int next = a.first_pass;
      if (!a.resume.empty()) next = r.load_checkpoint(a.resume, tag);
      const auto t0 = std::chrono::steady_clock::now();
      for (int done = next - a.first_pass; done < a.spp; done += a.chunk) {
        const int n = std::min(a.chunk, a.spp - done);
        r.render(cam, a.first_pass + done, n, a.date, a.bounces, a.ior, a.variant);
        kernel_ms += r.last_render_ms();
        if (!a.checkpoint.empty()) r.save_checkpoint(a.checkpoint, a.first_pass + done + n, tag);
      }
      img = r.read_image();
      wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    } else {
      // N shards: scene upload and targets first (untimed), then one host thread per shard
      const int N = (int)a.devices.size();
      std::vector<std::unique_ptr<mcpt::Renderer>> shards;
      for (int k = 0; k < N; ++k) {
        shards.emplace_back(new mcpt::Renderer(a.devices[(size_t)k]));
        shards.back()->set_traversal(a.traversal);
        shards.back()->upload(scene);
        shards.back()->set_target_rows(W, H, mcpt::Renderer::balanced_rows(H, N, k));
      }
      mcpt::Renderer frame(a.devices[0]);
      frame.set_target(W, H);
      std::vector<double> shard_ms((size_t)N, 0.0);
      std::vector<std::string> errors((size_t)N);
      const auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> workers;
      for (int k = 0; k < N; ++k)
        workers.emplace_back([&, k]() {
          try {
            for (int done = 0; done < a.spp; done += a.chunk) {
              const int n = std::min(a.chunk, a.spp - done);
              shards[(size_t)k]->render(cam, a.first_pass + done, n, a.date, a.bounces, a.ior, a.variant);
              shard_ms[(size_t)k] += shards[(size_t)k]->last_render_ms();   // (synchronizes this shard)
            }
          } catch (const std::exception& e) {
            errors[(size_t)k] = e.what();
          }
        });
      for (std::thread& t : workers) t.join();
      for (const std::string& e : errors)
        if (!e.empty()) throw std::runtime_error(e);
      const auto t1 = std::chrono::steady_clock::now();
      std::vector<const mcpt::Renderer*> views;
      for (const auto& r : shards) views.push_back(r.get());
      frame.gather_rows(views);
      img = frame.read_image();
      const auto t2 = std::chrono::steady_clock::now();
      wall_ms = std::chrono::duration<double, std::milli>(t2 - t0).count();
      gather_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
      for (double ms : shard_ms) kernel_ms = std::max(kernel_ms, ms);   // the slowest shard bounds the frame
      shard_json = ", \"devices\": [";
      for (int k = 0; k < N; ++k) shard_json += (k ? ", " : "") + std::to_string(a.devices[(size_t)k]);
      shard_json += "], \"shard_kernel_ms\": [";
      for (int k = 0; k < N; ++k) {
        char buf[32];
        std::snprintf(buf, sizeof(buf), "%s%.3f", k ? ", " : "", shard_ms[(size_t)k]);
        shard_json += buf;
      }
      char buf[64];
      std::snprintf(buf, sizeof(buf), "], \"gather_ms\": %.3f", gather_ms);
      shard_json += buf;
    }
    if (!a.pfm.empty()) mcpt::write_pfm(a.pfm, img, W, H);
    if (!a.png.empty()) mcpt::write_png(a.png, img, W, H);
    double mean = 0.0;
    for (float v : img) mean += v;
    mean /= (double)(img.size() ? img.size() : 1);
    const double samples = (double)W * H * a.spp;
    std::printf("{\"scene\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"bounces\": %d, \"ior\": %g, "
                "\"light\": %g, \"variant\": %d, \"prims\": %d, \"depth\": %d, \"kernel_ms\": %.3f, "
                "\"wall_ms\": %.3f, \"msamples_per_s\": %.2f, \"mean\": %.6f%s}\n",
                a.scene, W, H, a.spp, a.bounces, a.ior, a.light, a.variant, scene.nb_prim(), scene.depth(),
                kernel_ms, wall_ms, kernel_ms > 0 ? samples / kernel_ms / 1e3 : 0.0, mean, shard_json.c_str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mcpt_render: %s\n", e.what());
    return 1;
  }
  return 0;
}
