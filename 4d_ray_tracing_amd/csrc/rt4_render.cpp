// rt4_render — the reference's frame loop (src/main.cpp:57-111) offscreen, as a C++ host program over
// the C ABI of librt4.so: properties.txt + a scene .frag in, progressive frames of one section or of
// the three ThreeWindowGroup sections rendered on one GPU, PPM images out. What it replaces:
//   Properties props("properties.txt")            -> rt4_properties_load
//   initShader / initControls                     -> rt4_uniforms_from_properties / rt4_camera_init
//   shader.loadFromFile(shader_filename)          -> rt4_scene_load_frag (snippet or whole shader.frag)
//   seed ^= generateSeed(timer); part = 1/frame    -> seed ^ n*0x9E3779B9 (deterministic), camera uniforms
//   windowGroup->drawShaderImage()                -> rt4_render_sections_device (one launch, 1 or 3 images)
//   windowGroup->display()                        -> rt4_write_ppm after the last frame
// Usage: rt4_render [-p properties.txt] [-s scene(.frag|builtin name)] [-n frames] [-3] [-W width -H height]
//                   [-f f32|f16|rgba8] [--seed S] [-o prefix] [-d device] [--keys WASD...] [--move-seconds t]
//                   [--frame-by-frame]  (one section and a resting camera: rt4_render_frames_device unless given)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
  std::string props_path = "properties.txt", scene_arg, out = "frame", fmt_name = "f32";
  int frames = 1, device = 0, width = 0, height = 0;
  bool three = false, frame_by_frame = false;
  uint32_t seed = 12345, keys = 0;
  float move_seconds = 0.0f;
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

  rt4_context* ctx = nullptr;
  RT4_CHECK(rt4_context_create(device, RT4_FLAG_SAMPLER_LUT, &ctx, err, sizeof err));
  RT4_CHECK(rt4_context_set_scene(ctx, scene, err, sizeof err));
  const int32_t px = rt4_frame_format_bytes(format);
  void* d_frame[3] = {nullptr, nullptr, nullptr};
  for (int q = 0; q < n_img; q++) {
    HIP_CHECK(hipMalloc(&d_frame[q], static_cast<size_t>(cw[q]) * ch[q] * px));
    HIP_CHECK(hipMemset(d_frame[q], 0, static_cast<size_t>(cw[q]) * ch[q] * px));  // cleared RenderTexture
  }
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
    RT4_CHECK(rt4_context_reserve_frames(ctx, cw[0], ch[0], err, sizeof err));
    for (int n = 1; n <= frames; n++) {
      rt4_uniforms u;
      RT4_CHECK(rt4_camera_frame_uniforms(&cam, &base[0], sections[0],
                                          static_cast<int32_t>(seed ^ (static_cast<uint32_t>(n) * 0x9E3779B9u)), &u));
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
    const int32_t s_n = static_cast<int32_t>(seed ^ (static_cast<uint32_t>(n) * 0x9E3779B9u));
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
    const std::string path = out + "_" + names[q] + ".ppm";
    RT4_CHECK(rt4_write_ppm(path.c_str(), host.data(), format, cw[q], ch[q], cw[q], err, sizeof err));
    std::printf("wrote %s (%d x %d)\n", path.c_str(), cw[q], ch[q]);
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
