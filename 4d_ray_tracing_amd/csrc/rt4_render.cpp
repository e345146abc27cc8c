// rt4_render — the reference's frame loop (src/main.cpp:57-111) offscreen, as a C++ host program over
// the C ABI of librt4.so: properties.txt + a scene .frag in, progressive frames of one section or of
// the three ThreeWindowGroup sections rendered on one GPU, PPM images out. What it replaces:
//   Properties props("properties.txt")            -> rt4_properties_load
//   initShader / initControls                     -> rt4_uniforms_from_properties / rt4_camera_init
//   shader.loadFromFile(shader_filename)          -> rt4_scene_load_frag (snippet or whole shader.frag)
//   seed ^= generateSeed(timer); part = 1/frame    -> seed ^ n*0x9E3779B9 (deterministic), camera uniforms
//   windowGroup->drawShaderImage()                -> rt4_render_sections_device (one launch, 1 or 3 images)
//   windowGroup->display()                        -> rt4_write_ppm after the last frame
//   one GL draw of the whole texture (windows.cpp:45) -> with --gpus N: the frame's pixel bands over N GPUs,
//                                                    one host thread per device, each rank's frames in one
//                                                    rt4_render_frames_device call, one RCCL ncclGather of the
//                                                    padded shards to GPU 0 over xGMI, rt4_bands_unpermute_device
// Usage: rt4_render [-p properties.txt] [-s scene(.frag|builtin name)] [-n frames] [-3] [-W width -H height]
//                   [-f f32|f16|rgba8] [--seed S] [-o prefix] [-d device] [--keys WASD...] [--move-seconds t]
//                   [--frame-by-frame]  (one section and a resting camera: rt4_render_frames_device unless given)
//                   [--gpus N [--band B] [--rehearse]]  (one section, resting camera: bands over devices 0..N-1 +
//                   RCCL gather; --rehearse: N ranks on device 0, the gather as device copies, for one-GPU tests)
//                   [--png]  (PNG images instead of PPM)
//                   [--raw]  (also the frame's bytes as stored, <prefix>_<section>.raw: bit-exact comparisons)
//                   [--resume ckpt] [--checkpoint ckpt]  (one section: continue / save the progressive
//                   accumulator, rt4_accum_load / rt4_accum_save; the reference has no counterpart)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt4.h"

namespace {

[[noreturn]] void die(const char* what, const char* err) {
  std::fprintf(stderr, "rt4_render: %s: %s\n", what, err);
  std::exit(1);
}

#define RT4_CHECK(call)                       \
  do {                                        \
    if ((call) != RT4_OK) die(#call, err);    \
  } while (0)
#define HIP_CHECK(call)                                                 \
  do {                                                                  \
    hipError_t e_ = (call);                                             \
    if (e_ != hipSuccess) die(#call, hipGetErrorString(e_));            \
  } while (0)

// A reusable barrier for the device threads (C++17 has no std::barrier).
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  long gen_ = 0;
};

struct BandRun {  // one GPU's share of a --gpus run
  std::string error;
  unsigned long long count = 0;
  double ms = 0.0;  // this rank's wall time from the start barrier to its gather (and, on rank 0, the un-permute)
};

// Every rank's verdict on one step, agreed before anything collective runs: each rank posts its own
// result, waits at the barrier and reads them all (the barrier's mutex orders the posts before the reads).
// A rank that failed never leaves the others waiting in a collective, and no collective sees a null or
// partly set-up buffer: when any rank failed, every rank skips the gather and the un-permute.
class Agreement {
 public:
  Agreement(int n, Barrier& bar) : ok_(static_cast<size_t>(n), 1), bar_(bar) {}
  bool all(int rank, bool ok) {
    ok_[static_cast<size_t>(rank)] = ok ? 1 : 0;
    bar_.wait();
    bool all_ok = true;
    for (char v : ok_) all_ok = all_ok && v;
    bar_.wait();  // everyone has read before the next step posts again
    return all_ok;
  }

 private:
  std::vector<char> ok_;
  Barrier& bar_;
};

// The frames of one section on `gpus` devices: pixel bands dealt round-robin
// (rt4_band_plan), each rank's frames pipelined in one rt4_render_frames_device call into a padded
// shard of rows_max rows, one ncclGather of the shards to rank 0 and rt4_bands_unpermute_device there.
// The image equals a one-GPU render bit for bit (every pixel is independent: shader.frag:104-108).
//
// rehearse (--rehearse, a test switch for boxes with one GPU): every rank is a host thread with its own
// context, stream and buffers on device 0, and each rank copies its shard into its slot of rank 0's
// gathered buffer with hipMemcpyAsync where the real run calls ncclGather; the band plan, the barrier,
// the agreements and the un-permute are the real ones. fail_rank >= 0 (the RT4_RENDER_FAIL_RANK test hook)
// makes that rank's set-up fail after its allocations, or with fail_gather (RT4_RENDER_FAIL_STAGE=gather) its
// gather: the rank does not enqueue its part of the collective and reports an error, as when ncclGather fails.
// After the gather is enqueued the ranks agree once more: if any rank failed, every rank aborts its communicator
// (ncclCommAbort), so no rank waits forever in a collective its peer never joined. While the gather runs, every
// rank also watches its communicator's asynchronous error (ncclCommGetAsyncError) and a shared abort flag.
// Returns the frame on the host (rank 0's), or exits with status 1 naming the failed rank(s).
std::vector<unsigned char> render_bands(int gpus, int band, const rt4_scene_desc* scene, const std::vector<rt4_uniforms>& us,
                                        int32_t w, int32_t h, int32_t format, bool frame_by_frame, bool rehearse,
                                        int fail_rank, bool fail_gather, unsigned long long* count_out, double* ms_out) {
  const int32_t px = rt4_frame_format_bytes(format);
  std::vector<ncclComm_t> comms(static_cast<size_t>(gpus), nullptr);
  if (!rehearse) {
    std::vector<int> devs(static_cast<size_t>(gpus));
    for (int r = 0; r < gpus; r++) devs[static_cast<size_t>(r)] = r;
    if (ncclCommInitAll(comms.data(), gpus, devs.data()) != ncclSuccess) die("ncclCommInitAll", "failed");
  }
  std::vector<BandRun> runs(static_cast<size_t>(gpus));
  std::vector<unsigned char> image(static_cast<size_t>(w) * h * px);
  Barrier bar(gpus);
  Agreement agree(gpus, bar);
  void* root_gathered = nullptr;  // rank 0's gathered buffer (rehearse: the other ranks copy into it)
  std::atomic<bool> abort_all{false};  // a rank saw its communicator fail: every rank aborts its own
  auto rank_main = [&](int r) {
    BandRun& run = runs[static_cast<size_t>(r)];
    char err[1024] = {0};
    rt4_context* ctx = nullptr;
    void *shard = nullptr, *gathered = nullptr, *img = nullptr;
    unsigned long long* d_count = nullptr;
    hipStream_t stream = nullptr;
    rt4_region reg{0, 0, 0, 0, 0, 0};
    int32_t rows_max = 0;
    const int dev = rehearse ? 0 : r;
    auto fail = [&](const char* what) {
      if (run.error.empty()) run.error = what;
      return false;
    };
    bool ok = (hipSetDevice(dev) == hipSuccess && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess) ||
              fail("hipSetDevice / hipStreamCreate");
    if (ok && (rt4_band_plan(w, h, gpus, band, r, &reg, &rows_max, err, sizeof err) != RT4_OK ||
               rt4_context_create(dev, RT4_FLAG_SAMPLER_LUT, &ctx, err, sizeof err) != RT4_OK ||
               rt4_context_set_scene(ctx, scene, err, sizeof err) != RT4_OK))
      ok = fail(err);
    const size_t shard_bytes = static_cast<size_t>(rows_max) * w * px;
    if (ok) {
      ok = (hipMalloc(&shard, shard_bytes) == hipSuccess && hipMemset(shard, 0, shard_bytes) == hipSuccess &&
            hipMalloc(&d_count, sizeof *d_count) == hipSuccess && hipMemset(d_count, 0, sizeof *d_count) == hipSuccess) ||
           fail("device allocation");
      if (ok && r == 0)
        ok = (hipMalloc(&gathered, shard_bytes * gpus) == hipSuccess && hipMalloc(&img, image.size()) == hipSuccess) ||
             fail("device allocation");
    }
    const bool pipelined = ok && !frame_by_frame && us.size() >= 2 && reg.h > 0 &&
                           rt4_context_frames_per_launch(ctx, reg.w, reg.h) > 1;
    if (ok && pipelined && rt4_context_reserve_frames(ctx, reg.w, reg.h, err, sizeof err) != RT4_OK) ok = fail(err);
    if (ok && r == fail_rank && !fail_gather) ok = fail("set-up failure injected (RT4_RENDER_FAIL_RANK)");
    if (ok) ok = hipDeviceSynchronize() == hipSuccess || fail("hipDeviceSynchronize");
    if (r == 0) root_gathered = gathered;  // read by the other ranks only after the agreement's barrier
    // every rank set up (the agreement is also the start barrier): otherwise nobody renders or gathers
    const bool all_set = agree.all(r, ok);
    const auto t0 = std::chrono::steady_clock::now();
    if (all_set && reg.h > 0) {
      int st = RT4_OK;
      if (pipelined) {
        st = rt4_render_frames_device(ctx, us.data(), static_cast<int32_t>(us.size()), &reg, shard, format, w, d_count,
                                      stream, err, sizeof err);
      } else {
        for (size_t f = 0; f < us.size() && st == RT4_OK; f++)
          st = rt4_render_device_ex(ctx, &us[f], &reg, shard, format, w, d_count, stream, err, sizeof err);
      }
      if (st != RT4_OK) ok = fail(err);
    }
    // the renders were enqueued everywhere: only then the collective (a launch error skips it on every rank)
    const bool all_rendered = all_set && agree.all(r, ok);
    bool all_gathered = false;
    if (all_rendered) {
      ncclComm_t comm = rehearse ? nullptr : comms[static_cast<size_t>(r)];
      if (r == fail_rank && fail_gather) {
        ok = fail(rehearse ? "rehearsal gather copy failure injected (RT4_RENDER_FAIL_STAGE=gather)"
                           : "ncclGather failure injected (RT4_RENDER_FAIL_STAGE=gather)");
      } else if (rehearse) {
        ok = (hipMemcpyAsync(static_cast<char*>(root_gathered) + static_cast<size_t>(r) * shard_bytes, shard, shard_bytes,
                             hipMemcpyDeviceToDevice, stream) == hipSuccess &&
              hipStreamSynchronize(stream) == hipSuccess) ||
             fail("rehearsal gather copy");
      } else if (ncclGather(shard, gathered, shard_bytes, ncclUint8, 0, comm, stream) != ncclSuccess) {
        ok = fail("ncclGather failed");
      }
      // every rank enqueued its part (rehearse: every shard is in rank 0's buffer): otherwise the ranks that did
      // wait for a peer that never joins, so every rank aborts its communicator instead of synchronising
      all_gathered = agree.all(r, ok);
      if (!all_gathered) {
        abort_all = true;
      } else if (!rehearse) {
        // the gather runs: watch the communicator (an asynchronous error on any rank aborts them all)
        hipError_t q;
        while ((q = hipStreamQuery(stream)) == hipErrorNotReady && !abort_all) {
          ncclResult_t ae = ncclSuccess;
          if (ncclCommGetAsyncError(comm, &ae) != ncclSuccess || ae != ncclSuccess) {
            ok = fail("RCCL asynchronous error in ncclGather");
            abort_all = true;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
        if (q != hipSuccess && q != hipErrorNotReady) ok = fail("hipStreamQuery after ncclGather");
      }
      if (abort_all && comm) {
        (void)ncclCommAbort(comm);  // returns the pending collective; the communicator is gone
        comms[static_cast<size_t>(r)] = nullptr;
        if (ok) ok = fail("communicator aborted: another rank failed in the gather");
      }
      if (ok && !abort_all && r == 0 &&
          rt4_bands_unpermute_device(gathered, img, w, h, gpus, band, rows_max, format, stream, err, sizeof err) != RT4_OK)
        ok = fail(err);
    }
    if (stream && hipStreamSynchronize(stream) != hipSuccess && !abort_all) ok = fail("hipStreamSynchronize");
    run.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((!all_rendered || !all_gathered) && ok) fail("skipped: another rank failed");
    if (ok && hipMemcpy(&run.count, d_count, sizeof run.count, hipMemcpyDeviceToHost) != hipSuccess) fail("count");
    if (ok && r == 0 && hipMemcpy(image.data(), img, image.size(), hipMemcpyDeviceToHost) != hipSuccess)
      fail("image copy");
    if (shard) (void)hipFree(shard);
    if (gathered) (void)hipFree(gathered);
    if (img) (void)hipFree(img);
    if (d_count) (void)hipFree(d_count);
    if (stream) (void)hipStreamDestroy(stream);
    rt4_context_destroy(ctx);
  };
  std::vector<std::thread> threads;
  for (int r = 0; r < gpus; r++) threads.emplace_back(rank_main, r);
  for (auto& t : threads) t.join();
  for (auto& c : comms)
    if (c) (void)ncclCommDestroy(c);
  unsigned long long count = 0;
  double ms = 0.0;
  std::string errors;
  for (int r = 0; r < gpus; r++) {
    const BandRun& run = runs[static_cast<size_t>(r)];
    if (!run.error.empty()) errors += (errors.empty() ? "rank " : "; rank ") + std::to_string(r) + ": " + run.error;
    count += run.count;
    ms = std::max(ms, run.ms);  // the job's time: the slowest rank
  }
  if (!errors.empty()) die("--gpus", errors.c_str());
  *count_out = count;
  *ms_out = ms;
  return image;
}

void write_raw(const std::string& path, const std::vector<unsigned char>& bytes) {  // --raw
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) die("--raw", path.c_str());
  const bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
  if (std::fclose(f) != 0 || !ok) die("--raw: write failed", path.c_str());
}

uint32_t keys_from(const char* s) {  // controls.cpp:98-113 key names
  uint32_t k = 0;
  for (; *s; ++s) switch (*s) {
      case 'W': k |= RT4_KEY_FORWARD; break;
      case 'S': k |= RT4_KEY_BACK; break;
      case 'D': k |= RT4_KEY_RIGHT; break;
      case 'A': k |= RT4_KEY_LEFT; break;
      case ' ': case 'U': k |= RT4_KEY_UP; break;
      case 'L': k |= RT4_KEY_DOWN; break;
      case 'E': k |= RT4_KEY_W_POS; break;
      case 'Q': k |= RT4_KEY_W_NEG; break;
      default: break;
    }
  return k;
}

}  // namespace

int main(int argc, char** argv) {
  // The frame loop's overlapped launches of small frames use up to 8 side streams: give the
  // process 8 hardware queues unless the environment says otherwise (read when the HIP runtime starts).
  setenv("GPU_MAX_HW_QUEUES", "8", 0);
  std::string props_path = "properties.txt", scene_arg, out = "frame", fmt_name = "f32";
  int frames = 1, device = 0, width = 0, height = 0;
  bool three = false, frame_by_frame = false;
  int gpus = 0, band = 8;
  uint32_t seed = 12345, keys = 0;
  float move_seconds = 0.0f;
  std::string resume_path, checkpoint_path;
  bool png = false, rehearse = false, raw = false;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) die("missing value for", a.c_str());
      return argv[++i];
    };
    if (a == "-p") props_path = next();
    else if (a == "-s") scene_arg = next();
    else if (a == "-n") frames = std::atoi(next());
    else if (a == "-3") three = true;
    else if (a == "-W") width = std::atoi(next());
    else if (a == "-H") height = std::atoi(next());
    else if (a == "-f") fmt_name = next();
    else if (a == "--seed") seed = static_cast<uint32_t>(std::strtoul(next(), nullptr, 0));
    else if (a == "-o") out = next();
    else if (a == "-d") device = std::atoi(next());
    else if (a == "--keys") keys = keys_from(next());
    else if (a == "--frame-by-frame") frame_by_frame = true;
    else if (a == "--move-seconds") move_seconds = static_cast<float>(std::atof(next()));
    else if (a == "--gpus") gpus = std::atoi(next());
    else if (a == "--band") band = std::atoi(next());
    else if (a == "--resume") resume_path = next();
    else if (a == "--checkpoint") checkpoint_path = next();
    else if (a == "--png") png = true;
    else if (a == "--raw") raw = true;
    else if (a == "--rehearse") rehearse = true;
    else die("unknown argument", a.c_str());
  }
  const int32_t format = fmt_name == "f16" ? RT4_FRAME_RGBA16F : fmt_name == "rgba8" ? RT4_FRAME_RGBA8 : RT4_FRAME_RGBA32F;
  char err[1024] = {0};
  rt4_properties* props = nullptr;
  RT4_CHECK(rt4_properties_load(props_path.c_str(), &props, err, sizeof err));

  // scene: -s builtin name or .frag path; else the properties' shader_filename (main.cpp:26)
  rt4_scene_desc* scene = static_cast<rt4_scene_desc*>(std::calloc(1, sizeof(rt4_scene_desc)));
  if (scene_arg.empty()) {
    char buf[4096];
    size_t need = 0;
    RT4_CHECK(rt4_properties_get_string(props, "shader_filename", buf, sizeof buf, &need, err, sizeof err));
    scene_arg = buf;
  }
  if (scene_arg.size() > 5 && scene_arg.compare(scene_arg.size() - 5, 5, ".frag") == 0)
    RT4_CHECK(rt4_scene_load_frag(scene_arg.c_str(), scene, err, sizeof err));
  else
    RT4_CHECK(rt4_scene_builtin(scene_arg.c_str(), scene, err, sizeof err));

  // images: the main section (window.main cells, or -W/-H) and, with -3, YWZ / YXW (window.additional)
  const int n_img = three ? 3 : 1;
  int32_t cw[3], ch[3];
  if (width > 0 && height > 0) {
    cw[0] = width;
    ch[0] = height;
  } else {
    RT4_CHECK(rt4_window_cells(props, "main", &cw[0], &ch[0], err, sizeof err));
  }
  if (three) {
    RT4_CHECK(rt4_window_cells(props, "additional", &cw[1], &ch[1], err, sizeof err));
    cw[2] = cw[1];
    ch[2] = ch[1];
  }
  const int sections[3] = {RT4_SECTION_YXZ, RT4_SECTION_YWZ, RT4_SECTION_YXW};
  rt4_uniforms base[3];
  for (int q = 0; q < n_img; q++)
    RT4_CHECK(rt4_uniforms_from_properties(props, cw[q], ch[q], sections[q], &base[q], nullptr, err, sizeof err));
  rt4_camera cam;
  RT4_CHECK(rt4_camera_init(props, &cam, err, sizeof err));

  // the run's key, checked on --resume and recorded by --checkpoint: the first frame's uniforms (seed and
  // part aside they are every resting frame's)
  uint32_t run_key = 0;
  {
    rt4_camera c0 = cam;
    rt4_uniforms u0;
    RT4_CHECK(rt4_camera_frame_uniforms(&c0, &base[0], sections[0], 0, &u0));
    run_key = rt4_accum_key(scene, &u0);
  }
  if ((!resume_path.empty() || !checkpoint_path.empty()) && (three || gpus > 0))
    die("--resume/--checkpoint", "need one section on one GPU");
  // frames already blended into the accumulator (a resumed run continues at frame frames_done + 1)
  int64_t frames_done = 0;
  std::vector<unsigned char> resumed;
  if (!resume_path.empty()) {
    uint32_t ck_seed = 0;
    resumed.resize(static_cast<size_t>(cw[0]) * ch[0] * rt4_frame_format_bytes(format));
    RT4_CHECK(rt4_accum_load(resume_path.c_str(), resumed.data(), format, cw[0], ch[0], cw[0], &frames_done, &ck_seed, err,
                             sizeof err));
    if (ck_seed != seed) die("--resume", "the checkpoint was made with another --seed");
    // the checkpoint's run key (scene, samples, bounces, resolution, camera ...): a checkpoint of
    // another run would be blended in silently
    uint32_t ck_key = 0;
    RT4_CHECK(rt4_accum_key_of(resume_path.c_str(), &ck_key, err, sizeof err));
    if (ck_key != 0u && ck_key != run_key)
      die("--resume", "the checkpoint was made with another scene, properties or camera");
    cam.frame_number = static_cast<uint32_t>(frames_done + 1);
  }

  if (gpus > 0) {  // pixel bands over GPUs 0..gpus-1, one RCCL gather (one section, resting camera)
    if (three || (keys && move_seconds > 0.0f)) die("--gpus", "needs one section and a resting camera");
    if (frames < 1 || band < 1) die("--gpus", "frames and band must be >= 1");
    if (!rehearse) {  // a rehearsal puts every rank on device 0 and reports a missing device per rank
      int ndev = 0;
      HIP_CHECK(hipGetDeviceCount(&ndev));
      if (gpus > ndev) die("--gpus", ("only " + std::to_string(ndev) + " HIP devices").c_str());
    }
    const char* fail_env = std::getenv("RT4_RENDER_FAIL_RANK");  // test hook: this rank's set-up fails,
    const int fail_rank = fail_env ? std::atoi(fail_env) : -1;
    const char* stage_env = std::getenv("RT4_RENDER_FAIL_STAGE");  // or with "gather" its part of the gather
    const bool fail_gather = stage_env && std::strcmp(stage_env, "gather") == 0;
    std::vector<rt4_uniforms> us;
    for (int n = 1; n <= frames; n++) {
      rt4_uniforms u;
      RT4_CHECK(rt4_camera_frame_uniforms(&cam, &base[0], sections[0],
                                          static_cast<int32_t>(seed ^ (static_cast<uint32_t>(n) * 0x9E3779B9u)), &u));
      us.push_back(u);
    }
    unsigned long long count = 0;
    double ms = 0.0;
    const std::vector<unsigned char> img =
        render_bands(gpus, band, scene, us, cw[0], ch[0], format, frame_by_frame, rehearse, fail_rank, fail_gather, &count,
                     &ms);
    const std::string path = out + (png ? "_yxz.png" : "_yxz.ppm");
    RT4_CHECK((png ? rt4_write_png : rt4_write_ppm)(path.c_str(), img.data(), format, cw[0], ch[0], cw[0], err, sizeof err));
    if (raw) write_raw(out + "_yxz.raw", img);
    std::printf("wrote %s (%d x %d)\n", path.c_str(), cw[0], ch[0]);
    std::printf("gpus %d, frames %d, images 1, intersections %llu, %.3f ms/frame, %.3e intersections/s\n", gpus,
                frames, count, ms / frames, static_cast<double>(count) / (ms * 1e-3));
    rt4_properties_free(props);
    std::free(scene);
    return 0;
  }

  rt4_context* ctx = nullptr;
  RT4_CHECK(rt4_context_create(device, RT4_FLAG_SAMPLER_LUT, &ctx, err, sizeof err));
  RT4_CHECK(rt4_context_set_scene(ctx, scene, err, sizeof err));
  const int32_t px = rt4_frame_format_bytes(format);
  void* d_frame[3] = {nullptr, nullptr, nullptr};
  for (int q = 0; q < n_img; q++) {
    HIP_CHECK(hipMalloc(&d_frame[q], static_cast<size_t>(cw[q]) * ch[q] * px));
    HIP_CHECK(hipMemset(d_frame[q], 0, static_cast<size_t>(cw[q]) * ch[q] * px));  // cleared RenderTexture
  }
  if (!resumed.empty()) HIP_CHECK(hipMemcpy(d_frame[0], resumed.data(), resumed.size(), hipMemcpyHostToDevice));
  unsigned long long* d_count = nullptr;
  HIP_CHECK(hipMalloc(&d_count, sizeof *d_count));
  HIP_CHECK(hipMemset(d_count, 0, sizeof *d_count));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));

  // One section and a resting camera (progressive accumulation): the frames go to the library in one
  // rt4_render_frames_device call (pipelined through one pixel queue; the same final image).
  const bool pipelined = n_img == 1 && !(keys && move_seconds > 0.0f) && !frame_by_frame;
  std::vector<rt4_uniforms> us;
  if (pipelined) {
    // the frame-colour scratch only when frames are actually pipelined (>= 2 frames, a scene that does
    // not run frame by frame), and only for the frames of one chunk
    if (frames >= 2 && rt4_context_frames_per_launch(ctx, cw[0], ch[0]) > 1)
      RT4_CHECK(rt4_context_reserve_frames(ctx, cw[0], ch[0], err, sizeof err));
    for (int n = 1; n <= frames; n++) {
      rt4_uniforms u;
      const uint32_t fn = static_cast<uint32_t>(frames_done + n);
      RT4_CHECK(rt4_camera_frame_uniforms(&cam, &base[0], sections[0], static_cast<int32_t>(seed ^ (fn * 0x9E3779B9u)), &u));
      us.push_back(u);
    }
  }
  HIP_CHECK(hipEventRecord(e0, nullptr));
  if (pipelined) {
    const rt4_region reg{0, 0, cw[0], ch[0], 0, 0};
    RT4_CHECK(rt4_render_frames_device(ctx, us.data(), frames, &reg, d_frame[0], format, cw[0], d_count, nullptr, err,
                                       sizeof err));
  }
  for (int n = 1; n <= frames && !pipelined; n++) {
    const int32_t s_n = static_cast<int32_t>(seed ^ (static_cast<uint32_t>(frames_done + n) * 0x9E3779B9u));
    rt4_section_job jobs[3];
    const uint32_t frame_number = cam.frame_number;
    for (int q = 0; q < n_img; q++) {
      cam.frame_number = frame_number;  // one frame: every section gets the same part
      RT4_CHECK(rt4_camera_frame_uniforms(&cam, &base[q], sections[q], s_n, &jobs[q].u));
      jobs[q].region = rt4_region{0, 0, cw[q], ch[q], 0, 0};
      jobs[q].d_frame = d_frame[q];
      jobs[q].row_stride_px = cw[q];
    }
    RT4_CHECK(rt4_render_sections_device(ctx, jobs, n_img, format, d_count, nullptr, err, sizeof err));
    if (keys && move_seconds > 0.0f) rt4_camera_move(&cam, keys, move_seconds);  // move(seconds), main.cpp:95-96
  }
  HIP_CHECK(hipEventRecord(e1, nullptr));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.0f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long count = 0;
  HIP_CHECK(hipMemcpy(&count, d_count, sizeof count, hipMemcpyDeviceToHost));

  static const char* names[3] = {"yxz", "ywz", "yxw"};
  for (int q = 0; q < n_img; q++) {
    std::vector<unsigned char> host(static_cast<size_t>(cw[q]) * ch[q] * px);
    HIP_CHECK(hipMemcpy(host.data(), d_frame[q], host.size(), hipMemcpyDeviceToHost));
    const std::string path = out + "_" + names[q] + (png ? ".png" : ".ppm");
    RT4_CHECK((png ? rt4_write_png : rt4_write_ppm)(path.c_str(), host.data(), format, cw[q], ch[q], cw[q], err, sizeof err));
    if (raw) write_raw(out + "_" + names[q] + ".raw", host);
    std::printf("wrote %s (%d x %d)\n", path.c_str(), cw[q], ch[q]);
    if (q == 0 && !checkpoint_path.empty()) {
      // frames_done counts camera-resting frames only: a moving camera restarts the blend (frame_number 1)
      RT4_CHECK(rt4_accum_save_key(checkpoint_path.c_str(), host.data(), format, cw[0], ch[0], cw[0],
                                   static_cast<int64_t>(cam.frame_number) - 1, seed, run_key, err, sizeof err));
      std::printf("checkpoint %s (%lld frames)\n", checkpoint_path.c_str(), static_cast<long long>(cam.frame_number) - 1);
    }
  }
  std::printf("frames %d, images %d, intersections %llu, %.3f ms/frame, %.3e intersections/s\n", frames, n_img,
              count, ms / frames, static_cast<double>(count) / (ms * 1e-3));

  for (int q = 0; q < n_img; q++) (void)hipFree(d_frame[q]);
  (void)hipFree(d_count);
  rt4_context_destroy(ctx);
  rt4_properties_free(props);
  std::free(scene);
  return 0;
}
