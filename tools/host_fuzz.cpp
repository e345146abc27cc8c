// host_fuzz.cpp — sanitizer driver for librt4's host-side C++ (rt4_host.cpp: the scene .frag loader,
// the properties.txt parser, the camera controller, the PPM writer). Built and run by
// tests/test_host_sanitizers.py with -fsanitize=address,undefined (host code only, no GPU).
//
// Usage: host_fuzz <tmpdir> <file.frag|properties.txt>...
//   * every input parses (status 0) unmodified;
//   * every prefix of it, and 3000 seeded byte mutations of it, parse without a sanitizer report
//     (the status may be an error; the error text must be NUL-terminated within the buffer);
//   * the built-in scenes validate, the camera runs a scripted fly-through, PPM writes all formats.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../include/rt4.h"

namespace {

int failures = 0;
#define EXPECT(c)                                                                  \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #c); \
      failures++;                                                                  \
    }                                                                              \
  } while (0)

uint32_t rng_state = 0x9E3779B9u;
uint32_t next_u32() {  // xorshift32
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return rng_state;
}

bool is_properties(const std::string& path) { return path.size() >= 4 && path.compare(path.size() - 4, 4, ".txt") == 0; }

int parse(const std::string& path, const std::vector<char>& text) {
  char err[128];
  std::memset(err, 'x', sizeof err);
  // exact-size heap copy: a read past the end is an ASan report
  std::vector<char> buf(text);
  const char* ptr = buf.empty() ? "" : buf.data();
  int st;
  if (is_properties(path)) {
    rt4_properties* p = nullptr;
    st = rt4_properties_parse(ptr, buf.size(), &p, err, sizeof err);
    if (st == RT4_OK) {
      float f;
      int32_t i;
      char s[64];
      size_t need = 0;
      char e2[128];
      (void)rt4_properties_get_float(p, "camera.matrix_height", &f, e2, sizeof e2);
      (void)rt4_properties_get_int(p, "ray_tracing.samples", &i, e2, sizeof e2);
      (void)rt4_properties_get_string(p, "shader_filename", s, sizeof s, &need, e2, sizeof e2);
      rt4_uniforms u;
      rt4_orientation o;
      (void)rt4_uniforms_from_properties(p, 64, 40, 0, &u, &o, e2, sizeof e2);
      rt4_camera cam;
      if (rt4_camera_init(p, &cam, e2, sizeof e2) == RT4_OK) {
        rt4_camera_mouse_move(&cam, 17, -9, 400);
        rt4_camera_wheel(&cam, 1.0f);
        rt4_camera_move(&cam, 0xFFFFFFFFu, 0.25f);
        rt4_uniforms next;
        (void)rt4_camera_frame_uniforms(&cam, &u, 1, 7, &next);
      }
      rt4_properties_free(p);
    }
  } else {
    rt4_scene_desc* d = new rt4_scene_desc;
    st = rt4_scene_parse_frag(ptr, buf.size(), d, err, sizeof err);
    if (st == RT4_OK) (void)rt4_scene_validate(d, err, sizeof err);
    delete d;
  }
  if (st != RT4_OK) EXPECT(std::memchr(err, '\0', sizeof err) != nullptr);
  return st;
}

std::vector<char> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  return std::vector<char>(s.begin(), s.end());
}

void fuzz_file(const std::string& path) {
  const std::vector<char> text = read_file(path);
  EXPECT(!text.empty());
  const int st = parse(path, text);
  if (st != RT4_OK) std::fprintf(stderr, "%s: does not parse (status %d)\n", path.c_str(), st);
  EXPECT(st == RT4_OK);
  for (size_t n = 0; n < text.size(); n++) parse(path, std::vector<char>(text.begin(), text.begin() + static_cast<long>(n)));
  static const char tokens[] = "(){}[];,=.-+*/ \n\t0123456789eEfuxyzw_";
  for (int m = 0; m < 3000; m++) {
    std::vector<char> t = text;
    const int edits = 1 + static_cast<int>(next_u32() % 4);
    for (int e = 0; e < edits && !t.empty(); e++) {
      const size_t at = next_u32() % t.size();
      switch (next_u32() % 4) {
        case 0: t[at] = tokens[next_u32() % (sizeof tokens - 1)]; break;  // token-ish byte
        case 1: t[at] = static_cast<char>(next_u32() & 0xFF); break;      // any byte
        case 2: t.erase(t.begin() + static_cast<long>(at)); break;        // deletion
        default: {                                                        // duplication
          const char c = t[next_u32() % t.size()];
          t.insert(t.begin() + static_cast<long>(at), c);
        }
      }
    }
    parse(path, t);
  }
  std::printf("fuzzed %s (%zu bytes)\n", path.c_str(), text.size());
}

void builtins_and_ppm(const std::string& tmpdir) {
  char err[256];
  static const char* names[] = {"sphere", "room", "tiger", "cylinder4d", "hypercube"};  // the reference's five
  for (const char* n : names) {
    rt4_scene_desc* d = new rt4_scene_desc;
    EXPECT(rt4_scene_builtin(n, d, err, sizeof err) == RT4_OK);
    EXPECT(rt4_scene_validate(d, err, sizeof err) == RT4_OK);
    delete d;
  }
  rt4_scene_desc* d = new rt4_scene_desc;
  EXPECT(rt4_scene_builtin("no-such-scene", d, err, sizeof err) != RT4_OK);
  delete d;
  const int w = 13, h = 5, stride = 17;
  const int32_t formats[] = {RT4_FRAME_RGBA32F, RT4_FRAME_RGBA16F, RT4_FRAME_RGBA8};
  for (int32_t f : formats) {
    const int32_t bpp = rt4_frame_format_bytes(f);
    // exact size: the last row ends at its last pixel, not at the stride
    std::vector<unsigned char> frame((static_cast<size_t>(stride) * (h - 1) + w) * bpp);
    for (size_t i = 0; i < frame.size(); i++) frame[i] = static_cast<unsigned char>(i * 37u);
    const std::string out = tmpdir + "/fuzz_" + std::to_string(f) + ".ppm";
    EXPECT(rt4_write_ppm(out.c_str(), frame.data(), f, w, h, stride, err, sizeof err) == RT4_OK);
  }
  std::vector<unsigned char> one(16);
  EXPECT(rt4_write_ppm((tmpdir + "/no/such/dir.ppm").c_str(), one.data(), RT4_FRAME_RGBA8, 1, 1, 1, err, sizeof err) !=
         RT4_OK);
  rt4_uniforms base{}, out{};
  EXPECT(rt4_progressive_uniforms(&base, 0, &out) != RT4_OK);
  EXPECT(rt4_progressive_uniforms(&base, 3, &out) == RT4_OK);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <tmpdir> <file>...\n", argv[0]);
    return 2;
  }
  builtins_and_ppm(argv[1]);
  for (int i = 2; i < argc; i++) fuzz_file(argv[i]);
  if (failures) {
    std::fprintf(stderr, "%d expectation(s) failed\n", failures);
    return 1;
  }
  std::printf("host_fuzz ok\n");
  return 0;
}
