// rt4_host.cpp — host side of librt4.so: everything the reference's C++ host and GLSL compiler did
// around the trace kernel, re-done as plain C++ behind include/rt4.h.
//   * properties.txt parser          (src/properties.cpp:12-77, src/util/util.cpp:9-57)
//   * camera basis + uniform values   (src/controls.cpp:64-86,140-159, src/main.cpp:25-39,86-91,
//                                      src/windows/windows.cpp:6-13,24-47, src/util/math.cpp:6-29)
//   * scene loader for the GLSL subset used by scenes/<name>.frag and executable/shader.frag:412-468
//   * the reference's five scenes as built-ins
// Compiled with -ffp-contract=off: every fp32 expression is evaluated exactly as written.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include <unistd.h>  // fsync (rt4_accum_save_key)

#include "../../include/rt4.h"
#include "rt4_internal.h"

namespace {

constexpr float PI_F = 3.14159265f;      // inc/util/math.h:8, shader.frag:23
constexpr float GOLDEN_F = 1.61803399f;  // inc/util/math.h:9
constexpr float SMALL_F = 0.0003f;       // shader.frag:24

// ============================================================================ properties
std::string trim(const std::string& s, const char* ws = " \t") {  // util.cpp:39-45
  const auto b = s.find_first_not_of(ws);
  if (b == std::string::npos) return "";
  const auto e = s.find_last_not_of(ws);
  return s.substr(b, e - b + 1);
}

}  // namespace

struct rt4_properties {
  std::unordered_map<std::string, std::string> map;
};

namespace {

int parse_properties_text(const std::string& text, rt4_properties* p, char* err, size_t errlen) {
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {  // properties.cpp:17-27
    if (!line.empty() && line.back() == '\r') line.pop_back();  // CRLF files (the reference ran on Windows)
    const auto hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);  // takeBefore(line, "#")
    line = trim(line);
    if (line.empty()) continue;
    const auto eq = line.find('=');
    if (eq == std::string::npos) {
      rt4_set_err(err, errlen, "Failed to initialize properties. Cannot parse the line: \"%s\"", line.c_str());
      return RT4_ERR_PARSE;
    }
    // unordered_map::insert keeps the FIRST value of a repeated key (properties.cpp:25)
    p->map.insert({trim(line.substr(0, eq)), trim(line.substr(eq + 1))});
  }
  return RT4_OK;
}

const std::string* prop_find(const rt4_properties* p, const char* key, char* err, size_t errlen) {
  auto it = p->map.find(key);
  if (it == p->map.end()) {  // properties.cpp:35-38
    rt4_set_err(err, errlen, "Error! Cannot find property \"%s\".", key);
    return nullptr;
  }
  return &it->second;
}

}  // namespace

extern "C" {

int rt4_properties_parse(const char* text, size_t len, rt4_properties** out, char* err, size_t errlen) {
  if (!out || (!text && len)) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  *out = nullptr;
  auto* p = new rt4_properties();
  int st = parse_properties_text(std::string(text ? text : "", len), p, err, errlen);
  if (st != RT4_OK) {
    delete p;
    return st;
  }
  *out = p;
  return RT4_OK;
}

int rt4_properties_load(const char* path, rt4_properties** out, char* err, size_t errlen) {
  if (!path || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  *out = nullptr;
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {  // properties.cpp:29-30
    rt4_set_err(err, errlen, "Failed to initialize properties. Cannot open file \"%s\".", path);
    return RT4_ERR_IO;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  return rt4_properties_parse(s.data(), s.size(), out, err, errlen);
}

void rt4_properties_free(rt4_properties* p) { delete p; }

int rt4_properties_has(const rt4_properties* p, const char* key) {
  return (p && key && p->map.count(key)) ? 1 : 0;
}

int rt4_properties_get_string(const rt4_properties* p, const char* key, char* buf, size_t buflen, size_t* needed,
                              char* err, size_t errlen) {
  if (!p || !key) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const std::string* v = prop_find(p, key, err, errlen);
  if (!v) return RT4_ERR_PROPERTY;
  if (needed) *needed = v->size();
  if (buf && buflen) {
    const size_t n = v->size() < buflen - 1 ? v->size() : buflen - 1;
    std::memcpy(buf, v->data(), n);
    buf[n] = '\0';
  }
  return RT4_OK;
}

int rt4_properties_get_int(const rt4_properties* p, const char* key, int32_t* out, char* err, size_t errlen) {
  if (!p || !key || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const std::string* v = prop_find(p, key, err, errlen);
  if (!v) return RT4_ERR_PROPERTY;
  try {  // properties.cpp:43-50: std::stoi (leading integer, trailing text ignored)
    *out = std::stoi(*v);
  } catch (const std::invalid_argument&) {
    rt4_set_err(err, errlen, "Error! Cannot parse int value of property \"%s\".", key);
    return RT4_ERR_PROPERTY;
  } catch (const std::out_of_range&) {
    rt4_set_err(err, errlen, "Error! Value of property \"%s\" is out of the range.", key);
    return RT4_ERR_PROPERTY;
  }
  return RT4_OK;
}

int rt4_properties_get_uint(const rt4_properties* p, const char* key, uint32_t* out, char* err, size_t errlen) {
  if (!out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  int32_t v = 0;
  int st = rt4_properties_get_int(p, key, &v, err, errlen);
  if (st != RT4_OK) return st;
  if (v < 0) {  // properties.cpp:53-57
    rt4_set_err(err, errlen, "Error! Value of property \"%s\" must be positive.", key);
    return RT4_ERR_PROPERTY;
  }
  *out = static_cast<uint32_t>(v);
  return RT4_OK;
}

int rt4_properties_get_float(const rt4_properties* p, const char* key, float* out, char* err, size_t errlen) {
  if (!p || !key || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const std::string* v = prop_find(p, key, err, errlen);
  if (!v) return RT4_ERR_PROPERTY;
  std::stringstream stream(*v);  // properties.cpp:59-67: stringstream >> float
  float r;
  if (stream >> r) {
    *out = r;
    return RT4_OK;
  }
  rt4_set_err(err, errlen, "Error! Cannot parse float value of property \"%s\".", key);
  return RT4_ERR_PROPERTY;
}

int rt4_properties_get_bool(const rt4_properties* p, const char* key, int* out, char* err, size_t errlen) {
  if (!p || !key || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const std::string* v = prop_find(p, key, err, errlen);
  if (!v) return RT4_ERR_PROPERTY;
  std::string s = *v;  // properties.cpp:69-77: toLowerCase, "true" / "false"
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  if (s == "true") { *out = 1; return RT4_OK; }
  if (s == "false") { *out = 0; return RT4_OK; }
  rt4_set_err(err, errlen, "Error! Cannot parse boolean value of property \"%s\".", key);
  return RT4_ERR_PROPERTY;
}

// ============================================================================ camera + uniforms
static void rotate_pair(float angle, float* x, float* y) {  // controls.cpp:64-69
  const float sinA = std::sin(angle), cosA = std::cos(angle);
  float ox[4], oy[4];
  std::memcpy(ox, x, sizeof ox);
  std::memcpy(oy, y, sizeof oy);
  for (int k = 0; k < 4; k++) {
    x[k] = ox[k] * cosA + oy[k] * sinA;     // sum(mulVN(oldX, cosA), mulVN(oldY, sinA))
    y[k] = ox[k] * -sinA + oy[k] * cosA;    // sum(mulVN(oldX, -sinA), mulVN(oldY, cosA))
  }
}

void rt4_orientation_update(float fi, float te, float psi, rt4_orientation* o) {  // controls.cpp:72-86
  if (!o) return;
  const float fwd[4] = {0, 1, 0, 0}, top[4] = {0, 0, 1, 0}, right[4] = {1, 0, 0, 0}, w[4] = {0, 0, 0, 1};
  std::memcpy(o->forward, fwd, sizeof fwd);
  std::memcpy(o->top, top, sizeof top);
  std::memcpy(o->right, right, sizeof right);
  std::memcpy(o->w_drct, w, sizeof w);
  rotate_pair(psi, o->top, o->w_drct);
  std::memcpy(o->vertical_top, o->top, sizeof top);
  rotate_pair(fi, o->forward, o->right);
  std::memcpy(o->horizontal_forward, o->forward, sizeof fwd);
  std::memcpy(o->horizontal_right, o->right, sizeof right);
  rotate_pair(te, o->forward, o->top);
}

int rt4_section_basis(const rt4_orientation* o, int section, float top[4], float right[4]) {
  if (!o || !top || !right) return RT4_ERR_ARG;
  const float *t, *r;
  switch (section) {  // three_window_group.cpp:42-46
    case RT4_SECTION_YXZ: t = o->top; r = o->right; break;
    case RT4_SECTION_YWZ: t = o->top; r = o->w_drct; break;
    case RT4_SECTION_YXW: t = o->w_drct; r = o->right; break;
    default: return RT4_ERR_ARG;
  }
  std::memcpy(top, t, 4 * sizeof(float));
  std::memcpy(right, r, 4 * sizeof(float));
  return RT4_OK;
}

static void normalize_angle(float& a) {  // math.cpp:24-28
  a = std::remainder(a, 2 * PI_F);
  if (a < -PI_F) a += 2 * PI_F;
  if (a > PI_F) a -= 2 * PI_F;
}
static void pull_into_range(float& f, float center, float r) {  // math.cpp:19-22
  if (f < center - r) f = center - r;
  if (f > center + r) f = center + r;
}
static float deg2rad(float d) { return d / 180 * PI_F; }  // math.cpp:29

#define RT4_GETF(key, dst)                                               \
  do {                                                                   \
    int st_ = rt4_properties_get_float(p, key, &(dst), err, errlen);     \
    if (st_ != RT4_OK) return st_;                                       \
  } while (0)

int rt4_uniforms_from_properties(const rt4_properties* p, int32_t cells_w, int32_t cells_h, int section,
                                 rt4_uniforms* u, rt4_orientation* orientation_out, char* err, size_t errlen) {
  if (!p || !u) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (cells_w <= 0 || cells_h <= 0) return rt4_set_err(err, errlen, "resolution must be positive"), RT4_ERR_ARG;
  rt4_uniforms r;
  std::memset(&r, 0, sizeof r);
  uint32_t samples = 0, refl = 0;
  int st = rt4_properties_get_uint(p, "ray_tracing.samples", &samples, err, errlen);  // main.cpp:28
  if (st != RT4_OK) return st;
  st = rt4_properties_get_uint(p, "ray_tracing.reflections_amount", &refl, err, errlen);  // main.cpp:29
  if (st != RT4_OK) return st;
  r.samples = static_cast<int32_t>(samples);
  r.reflections_amount = static_cast<int32_t>(refl);
  RT4_GETF("ray_tracing.small_indent", r.small_indent);                                // main.cpp:30
  RT4_GETF("light_to_color_conversion_coefficient", r.light_to_color_conversion_coefficient);  // main.cpp:32-35
  float mtr_h = 0;
  RT4_GETF("camera.matrix_height", mtr_h);  // main.cpp:37-38
  r.mtr_sizes[0] = mtr_h * GOLDEN_F;
  r.mtr_sizes[1] = mtr_h;
  float focus_dist = 0;
  RT4_GETF("camera.focus_to_matrix_distance", focus_dist);  // main.cpp:73
  // initControls, controls.cpp:151-158
  RT4_GETF("camera.initial_position.x", r.focus[0]);
  RT4_GETF("camera.initial_position.y", r.focus[1]);
  RT4_GETF("camera.initial_position.z", r.focus[2]);
  RT4_GETF("camera.initial_position.w", r.focus[3]);
  float fi = 0, te = 0, psi = 0;
  RT4_GETF("camera.initial_position.fi", fi);
  RT4_GETF("camera.initial_position.te", te);
  RT4_GETF("camera.initial_position.psi", psi);
  fi = deg2rad(fi);  // SphOrientation::init, controls.cpp:29-39
  te = deg2rad(te);
  psi = deg2rad(psi);
  int constrain = 0;
  if (rt4_properties_has(p, "constrain_psi_range")) {
    st = rt4_properties_get_bool(p, "constrain_psi_range", &constrain, err, errlen);
    if (st != RT4_OK) return st;
  }
  float psi_center = 0, psi_radius = 0;
  if (constrain) {
    psi_center = psi;
    normalize_angle(psi_center);
    float deg = 0;
    RT4_GETF("psi_range_radius", deg);
    psi_radius = deg2rad(deg);
  }
  normalize_angle(fi);                 // normalizeFi
  pull_into_range(te, 0, PI_F / 2);    // normalizeTe
  if (constrain)                       // normalizePsi
    pull_into_range(psi, psi_center, psi_radius);
  else
    normalize_angle(psi);
  rt4_orientation o;
  rt4_orientation_update(fi, te, psi, &o);
  for (int k = 0; k < 4; k++) r.vec_to_mtr[k] = o.forward[k] * focus_dist;  // mulVN(forward, d), main.cpp:90
  if (rt4_section_basis(&o, section, r.top_drct, r.right_drct) != RT4_OK)
    return rt4_set_err(err, errlen, "bad section %d", section), RT4_ERR_ARG;
  r.resolution[0] = static_cast<float>(cells_w);  // windows.cpp:41
  r.resolution[1] = static_cast<float>(cells_h);
  r.part = 1.0f / 1;  // frameNumber = 1 (main.cpp:72,87)
  r.seed = 0;
  *u = r;
  if (orientation_out) *orientation_out = o;
  return RT4_OK;
}

int rt4_window_cells(const rt4_properties* p, const char* window_type, int32_t* cells_w, int32_t* cells_h, char* err,
                     size_t errlen) {
  if (!p || !window_type || !cells_w || !cells_h) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const std::string base = std::string("window.") + window_type + ".";
  uint32_t width = 0, cell = 0;
  int st = rt4_properties_get_uint(p, (base + "width").c_str(), &width, err, errlen);  // windows.cpp:10
  if (st != RT4_OK) return st;
  st = rt4_properties_get_uint(p, (base + "cell_size").c_str(), &cell, err, errlen);  // windows.cpp:12
  if (st != RT4_OK) return st;
  if (cell == 0) return rt4_set_err(err, errlen, "cell_size must be > 0"), RT4_ERR_PROPERTY;
  const unsigned height = static_cast<unsigned>(width / GOLDEN_F);  // windows.cpp:11 (unsigned member)
  *cells_w = static_cast<int32_t>(width / cell);                    // windows.cpp:25-26
  *cells_h = static_cast<int32_t>(height / cell);
  return RT4_OK;
}

// ============================================================================ camera (controls.cpp)
namespace {

float rt4_half_to_float(uint16_t h) {  // IEEE binary16 -> binary32 (exact)
  const uint32_t sign = static_cast<uint32_t>(h & 0x8000u) << 16, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
  uint32_t bits;
  if (e == 0) {
    float f = static_cast<float>(m) * 5.9604644775390625e-8f;  // m * 2^-24 (zero or subnormal)
    std::memcpy(&bits, &f, 4);
    bits |= sign;
  } else if (e == 31) {
    bits = sign | 0x7F800000u | (m << 13);
  } else {
    bits = sign | ((e + 112u) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

void camera_normalize(rt4_camera* c) {  // SphOrientation::normalize, controls.cpp:41-50
  normalize_angle(c->fi);
  pull_into_range(c->te, 0, PI_F / 2);
  if (c->constrain_psi_range)
    pull_into_range(c->psi, c->psi_range_center, c->psi_range_radius);
  else
    normalize_angle(c->psi);
}

}  // namespace

int rt4_camera_init(const rt4_properties* p, rt4_camera* cam, char* err, size_t errlen) {
  if (!p || !cam) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  rt4_camera c;
  std::memset(&c, 0, sizeof c);
  RT4_GETF("mouse_sensitivity", c.mouse_sensitivity);  // controls.cpp:145-147
  RT4_GETF("wheel_sensitivity", c.wheel_sensitivity);
  RT4_GETF("movement_speed", c.movement_speed);
  RT4_GETF("camera.focus_to_matrix_distance", c.focus_to_matrix_distance);  // main.cpp:73
  RT4_GETF("camera.initial_position.x", c.focus[0]);                        // controls.cpp:150-156
  RT4_GETF("camera.initial_position.y", c.focus[1]);
  RT4_GETF("camera.initial_position.z", c.focus[2]);
  RT4_GETF("camera.initial_position.w", c.focus[3]);
  RT4_GETF("camera.initial_position.fi", c.fi);  // SphOrientation::init, controls.cpp:29-39
  RT4_GETF("camera.initial_position.te", c.te);
  RT4_GETF("camera.initial_position.psi", c.psi);
  c.fi = deg2rad(c.fi);
  c.te = deg2rad(c.te);
  c.psi = deg2rad(c.psi);
  int constrain = 0;
  int st = rt4_properties_get_bool(p, "constrain_psi_range", &constrain, err, errlen);
  if (st != RT4_OK) return st;
  c.constrain_psi_range = constrain;
  if (constrain) {
    c.psi_range_center = c.psi;
    normalize_angle(c.psi_range_center);
    float deg = 0;
    RT4_GETF("psi_range_radius", deg);
    c.psi_range_radius = deg2rad(deg);
  }
  camera_normalize(&c);
  rt4_orientation_update(c.fi, c.te, c.psi, &c.orientation);
  c.frame_number = 1;
  *cam = c;
  return RT4_OK;
}

void rt4_camera_rotate(rt4_camera* cam, float d_fi, float d_te, float d_psi) {
  if (!cam) return;
  if (d_fi != 0.0f) { cam->fi += d_fi; normalize_angle(cam->fi); }                      // changeFi
  if (d_te != 0.0f) { cam->te += d_te; pull_into_range(cam->te, 0, PI_F / 2); }          // changeTe
  if (d_psi != 0.0f) {                                                                  // changePsi
    cam->psi += d_psi;
    if (cam->constrain_psi_range) pull_into_range(cam->psi, cam->psi_range_center, cam->psi_range_radius);
    else normalize_angle(cam->psi);
  }
  rt4_orientation_update(cam->fi, cam->te, cam->psi, &cam->orientation);
  cam->frame_number = 1;
}

int rt4_camera_mouse_move(rt4_camera* cam, int32_t dx, int32_t dy, uint32_t max_offset) {
  if (!cam) return 0;
  if (static_cast<uint32_t>(std::abs(dx)) > max_offset || static_cast<uint32_t>(std::abs(dy)) > max_offset)
    return 1;  // centerMouseCursor() only (controls.cpp:185-186)
  if (dx == 0 && dy == 0) return 0;
  rt4_camera_rotate(cam, static_cast<float>(dx) * cam->mouse_sensitivity, static_cast<float>(dy) * cam->mouse_sensitivity,
                    0.0f);
  return 0;
}

void rt4_camera_wheel(rt4_camera* cam, float delta) {
  if (!cam) return;
  rt4_camera_rotate(cam, 0.0f, 0.0f, delta * cam->wheel_sensitivity);
  cam->frame_number = 1;  // also when a constrained psi did not change (controls.cpp:199)
}

void rt4_camera_move(rt4_camera* cam, uint32_t keys, float seconds) {  // controls.cpp:118-134
  if (!cam) return;
  const rt4_orientation& o = cam->orientation;
  float d[4] = {0, 0, 0, 0};
  auto add = [&](const float* v, float sgn) {  // sum(drct, v) / dif(drct, v) = sum(drct, mulVN(v, -1))
    for (int k = 0; k < 4; k++) d[k] = d[k] + v[k] * sgn;
  };
  if (keys & RT4_KEY_FORWARD) add(o.horizontal_forward, 1.0f);
  if (keys & RT4_KEY_BACK) add(o.horizontal_forward, -1.0f);
  if (keys & RT4_KEY_UP) add(o.vertical_top, 1.0f);
  if (keys & RT4_KEY_DOWN) add(o.vertical_top, -1.0f);
  if (keys & RT4_KEY_RIGHT) add(o.horizontal_right, 1.0f);
  if (keys & RT4_KEY_LEFT) add(o.horizontal_right, -1.0f);
  if (keys & RT4_KEY_W_POS) add(o.w_drct, 1.0f);
  if (keys & RT4_KEY_W_NEG) add(o.w_drct, -1.0f);
  const float len = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);  // mod(), math.cpp:12-13
  if (len > 0) {
    const float k = seconds * cam->movement_speed / len;
    for (int q = 0; q < 4; q++) cam->focus[q] = cam->focus[q] + d[q] * k;
    cam->frame_number = 1;
  }
}

int rt4_camera_frame_uniforms(rt4_camera* cam, const rt4_uniforms* base, int section, int32_t seed,
                              rt4_uniforms* out) {
  if (!cam || !base || !out || cam->frame_number == 0) return RT4_ERR_ARG;
  rt4_uniforms u = *base;
  u.seed = seed;                                                 // main.cpp:86
  u.part = 1.0f / static_cast<float>(cam->frame_number);         // main.cpp:87
  std::memcpy(u.focus, cam->focus, sizeof u.focus);              // main.cpp:89
  for (int k = 0; k < 4; k++) u.vec_to_mtr[k] = cam->orientation.forward[k] * cam->focus_to_matrix_distance;  // :90
  if (rt4_section_basis(&cam->orientation, section, u.top_drct, u.right_drct) != RT4_OK) return RT4_ERR_ARG;
  cam->frame_number++;                                           // frameNumber++ (main.cpp:88)
  *out = u;
  return RT4_OK;
}

// ============================================================================ multi-GPU pixel bands
// Bands of `band` rows dealt round-robin over the ranks (shard.py make_plan is the same
// arithmetic, tests/test_shard.py compares the two). Band b holds image rows [b band, min((b+1) band, H))
// and belongs to rank b mod world; the rank's local row i is image row
// (i / band) band world + rank band + i mod band, the rt4_region band layout with y0 = rank band.
int rt4_band_plan(int32_t width, int32_t height, int32_t world, int32_t band, int32_t rank, rt4_region* region,
                  int32_t* rows_max, char* err, size_t errlen) {
  if (!region || !rows_max) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (width < 1 || height < 1 || world < 1 || band < 1)
    return rt4_set_err(err, errlen, "band plan: width %d, height %d, world %d, band %d must be >= 1", width, height,
                       world, band),
           RT4_ERR_ARG;
  if (rank < 0 || rank >= world) return rt4_set_err(err, errlen, "rank %d not in [0, %d)", rank, world), RT4_ERR_ARG;
  *rows_max = static_cast<int32_t>(rt4_band_rows_max(height, world, band));
  if (world == 1) {
    *region = rt4_region{0, 0, width, height, 0, 0};
  } else {
    *region = rt4_region{0, rank * band, width, static_cast<int32_t>(rt4_band_rows(height, world, band, rank)), band,
                         band * world};
  }
  return RT4_OK;
}

// ============================================================================ image output
namespace {
// One frame row as 8-bit RGB with the RGBA8 rule of rt4_frame_format (float channels clamped to [0, 1],
// u = (uint8)(v * 255 + 0.5)); shared by the PPM and PNG writers.
void rgb8_row(const void* frame, int32_t format, int32_t px_bytes, int32_t w, int64_t row_stride_px, int32_t i,
              unsigned char* row) {
  auto q8 = [](float v) {
    return static_cast<unsigned char>(static_cast<uint32_t>(std::fmin(std::fmax(v, 0.0f), 1.0f) * 255.0f + 0.5f));
  };
  const unsigned char* base = static_cast<const unsigned char*>(frame) + static_cast<size_t>(i) * row_stride_px * px_bytes;
  for (int32_t j = 0; j < w; j++) {
    const unsigned char* px = base + static_cast<size_t>(j) * px_bytes;
    for (int c = 0; c < 3; c++) {
      unsigned char v;
      if (format == RT4_FRAME_RGBA8) {
        v = px[c];
      } else if (format == RT4_FRAME_RGBA16F) {
        uint16_t hb;
        std::memcpy(&hb, px + 2 * c, 2);
        v = q8(rt4_half_to_float(hb));
      } else {
        float fv;
        std::memcpy(&fv, px + 4 * c, 4);
        v = q8(fv);
      }
      row[static_cast<size_t>(j) * 3 + c] = v;
    }
  }
}

uint32_t crc32_png(const unsigned char* p, size_t n, uint32_t c = 0xFFFFFFFFu) {  // PNG / zlib CRC-32
  for (size_t k = 0; k < n; k++) {
    c ^= p[k];
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return c;
}
void put_be32(std::vector<unsigned char>& v, uint32_t x) {
  for (int s = 24; s >= 0; s -= 8) v.push_back(static_cast<unsigned char>(x >> s));
}
bool png_chunk(std::FILE* f, const char* type, const std::vector<unsigned char>& data) {
  std::vector<unsigned char> buf;
  put_be32(buf, static_cast<uint32_t>(data.size()));
  buf.insert(buf.end(), type, type + 4);
  buf.insert(buf.end(), data.begin(), data.end());
  put_be32(buf, crc32_png(buf.data() + 4, buf.size() - 4) ^ 0xFFFFFFFFu);
  return std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
}
}  // namespace

int rt4_write_ppm(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                  char* err, size_t errlen) {
  if (!path || !frame || w <= 0 || h <= 0 || row_stride_px < w)
    return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  const int32_t px_bytes = rt4_frame_format_bytes(format);
  if (px_bytes == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  std::FILE* f = std::fopen(path, "wb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s for writing", path), RT4_ERR_IO;
  std::fprintf(f, "P6\n%d %d\n255\n", w, h);
  std::vector<unsigned char> row(static_cast<size_t>(w) * 3);
  for (int32_t i = 0; i < h; i++) {
    rgb8_row(frame, format, px_bytes, w, row_stride_px, i, row.data());
    if (std::fwrite(row.data(), 1, row.size(), f) != row.size()) {
      std::fclose(f);
      return rt4_set_err(err, errlen, "write failed: %s", path), RT4_ERR_IO;
    }
  }
  if (std::fclose(f) != 0) return rt4_set_err(err, errlen, "close failed: %s", path), RT4_ERR_IO;
  return RT4_OK;
}

int rt4_write_png(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                  char* err, size_t errlen) {
  if (!path || !frame || w <= 0 || h <= 0 || row_stride_px < w || static_cast<int64_t>(w) * 3 + 1 > 65535)
    return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  const int32_t px_bytes = rt4_frame_format_bytes(format);
  if (px_bytes == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  // 8-bit RGB, filter 0 on every row, zlib stream of stored (uncompressed) deflate blocks: one block per row
  // (a row of w * 3 + 1 bytes fits a stored block's 65535-byte limit), then Adler-32
  const size_t rb = static_cast<size_t>(w) * 3 + 1;
  std::vector<unsigned char> z = {0x78, 0x01};
  uint32_t a1 = 1, a2 = 0;
  std::vector<unsigned char> row(rb);
  for (int32_t i = 0; i < h; i++) {
    row[0] = 0;
    rgb8_row(frame, format, px_bytes, w, row_stride_px, i, row.data() + 1);
    z.push_back(i + 1 == h ? 1 : 0);  // BFINAL, BTYPE 00
    z.push_back(static_cast<unsigned char>(rb & 0xFF));
    z.push_back(static_cast<unsigned char>(rb >> 8));
    z.push_back(static_cast<unsigned char>(~rb & 0xFF));
    z.push_back(static_cast<unsigned char>((~rb >> 8) & 0xFF));
    z.insert(z.end(), row.begin(), row.end());
    for (unsigned char c : row) {
      a1 = (a1 + c) % 65521u;
      a2 = (a2 + a1) % 65521u;
    }
  }
  put_be32(z, (a2 << 16) | a1);
  std::vector<unsigned char> ihdr;
  put_be32(ihdr, static_cast<uint32_t>(w));
  put_be32(ihdr, static_cast<uint32_t>(h));
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8 bits, RGB, deflate, filter 0, no interlace
  std::FILE* f = std::fopen(path, "wb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s for writing", path), RT4_ERR_IO;
  static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  bool ok = std::fwrite(sig, 1, 8, f) == 8 && png_chunk(f, "IHDR", ihdr) && png_chunk(f, "IDAT", z) &&
            png_chunk(f, "IEND", {});
  if (std::fclose(f) != 0) ok = false;
  if (!ok) return rt4_set_err(err, errlen, "write failed: %s", path), RT4_ERR_IO;
  return RT4_OK;
}

// ============================================================================ accumulator checkpoint
namespace {
constexpr char kAccMagic[8] = {'R', 'T', '4', 'A', 'C', 'C', '1', '\0'};
struct AccHeader {  // the file's first 40 bytes (rt4.h), little-endian like every supported host
  char magic[8];
  int32_t version, w, h, format;
  int64_t frames_done;
  uint32_t seed, key;  // key: rt4_accum_key of the run (version 2; 0 = not recorded, as in version 1 files)
};
static_assert(sizeof(AccHeader) == 40, "checkpoint header layout");

int acc_read_header(std::FILE* f, const char* path, AccHeader& hd, char* err, size_t errlen) {
  if (std::fread(&hd, 1, sizeof hd, f) != sizeof hd || std::memcmp(hd.magic, kAccMagic, sizeof kAccMagic) != 0)
    return rt4_set_err(err, errlen, "%s is not an rt4 accumulator checkpoint", path), RT4_ERR_PARSE;
  if (hd.version != 1 && hd.version != RT4_ACCUM_VERSION)
    return rt4_set_err(err, errlen, "%s: checkpoint version %d, expected 1 or %d", path, hd.version, RT4_ACCUM_VERSION),
           RT4_ERR_PARSE;
  if (hd.version == 1) hd.key = 0;
  if (hd.w <= 0 || hd.h <= 0 || rt4_frame_format_bytes(hd.format) == 0 || hd.frames_done < 0)
    return rt4_set_err(err, errlen, "%s: bad checkpoint header", path), RT4_ERR_PARSE;
  return RT4_OK;
}
}  // namespace

// FNV-1a over the bytes that decide a progressive run's image besides seed and part: the scene and the
// uniforms' samples, bounces, indent, tone-map coefficient, resolution, matrix and camera pose
uint32_t rt4_accum_key(const rt4_scene_desc* scene, const rt4_uniforms* u) {
  uint32_t hsh = 2166136261u;
  auto mix = [&](const void* p, size_t n) {
    for (size_t i = 0; i < n; i++) hsh = (hsh ^ static_cast<const unsigned char*>(p)[i]) * 16777619u;
  };
  if (scene) mix(scene, sizeof *scene);
  if (u) {
    rt4_uniforms v = *u;
    v.seed = 0;
    v.part = 0.0f;
    mix(&v, sizeof v);
  }
  return hsh == 0u ? 1u : hsh;  // 0 means "not recorded"
}

int rt4_accum_save_key(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                       int64_t frames_done, uint32_t seed, uint32_t key, char* err, size_t errlen) {
  if (!path || !frame || w <= 0 || h <= 0 || row_stride_px < w || frames_done < 0)
    return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  const int32_t px_bytes = rt4_frame_format_bytes(format);
  if (px_bytes == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  AccHeader hd{};
  std::memcpy(hd.magic, kAccMagic, sizeof kAccMagic);
  hd.version = RT4_ACCUM_VERSION;
  hd.w = w;
  hd.h = h;
  hd.format = format;
  hd.frames_done = frames_done;
  hd.seed = seed;
  hd.key = key;
  // written next to the target, flushed to the disk, then renamed over it: a crash or a full disk
  // mid-write leaves the previous checkpoint intact
  const std::string tmp = std::string(path) + ".tmp";
  std::FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s for writing", tmp.c_str()), RT4_ERR_IO;
  bool ok = std::fwrite(&hd, 1, sizeof hd, f) == sizeof hd;
  const size_t row = static_cast<size_t>(w) * px_bytes;
  for (int32_t i = 0; ok && i < h; i++)
    ok = std::fwrite(static_cast<const unsigned char*>(frame) + static_cast<size_t>(i) * row_stride_px * px_bytes, 1,
                     row, f) == row;
  ok = ok && std::fflush(f) == 0 && fsync(fileno(f)) == 0;
  if (std::fclose(f) != 0) ok = false;
  if (ok && std::rename(tmp.c_str(), path) != 0) ok = false;
  if (!ok) {
    std::remove(tmp.c_str());
    return rt4_set_err(err, errlen, "write failed: %s", path), RT4_ERR_IO;
  }
  return RT4_OK;
}

int rt4_accum_save(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                   int64_t frames_done, uint32_t seed, char* err, size_t errlen) {
  return rt4_accum_save_key(path, frame, format, w, h, row_stride_px, frames_done, seed, 0u, err, errlen);
}

int rt4_accum_key_of(const char* path, uint32_t* key, char* err, size_t errlen) {
  if (!path || !key) return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  std::FILE* f = std::fopen(path, "rb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s", path), RT4_ERR_IO;
  AccHeader hd{};
  const int rc = acc_read_header(f, path, hd, err, errlen);
  std::fclose(f);
  if (rc == RT4_OK) *key = hd.key;
  return rc;
}

int rt4_accum_info(const char* path, int32_t* w, int32_t* h, int32_t* format, int64_t* frames_done, uint32_t* seed,
                   char* err, size_t errlen) {
  if (!path) return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  std::FILE* f = std::fopen(path, "rb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s", path), RT4_ERR_IO;
  AccHeader hd{};
  const int rc = acc_read_header(f, path, hd, err, errlen);
  std::fclose(f);
  if (rc != RT4_OK) return rc;
  if (w) *w = hd.w;
  if (h) *h = hd.h;
  if (format) *format = hd.format;
  if (frames_done) *frames_done = hd.frames_done;
  if (seed) *seed = hd.seed;
  return RT4_OK;
}

int rt4_accum_load(const char* path, void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                   int64_t* frames_done, uint32_t* seed, char* err, size_t errlen) {
  if (!path || !frame || w <= 0 || h <= 0 || row_stride_px < w) return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  std::FILE* f = std::fopen(path, "rb");
  if (!f) return rt4_set_err(err, errlen, "cannot open %s", path), RT4_ERR_IO;
  AccHeader hd{};
  int rc = acc_read_header(f, path, hd, err, errlen);
  if (rc == RT4_OK && (hd.w != w || hd.h != h || hd.format != format)) {
    rt4_set_err(err, errlen, "%s holds a %dx%d frame of format %d, not %dx%d of format %d", path, hd.w, hd.h, hd.format,
                w, h, format);
    rc = RT4_ERR_ARG;
  }
  const int32_t px_bytes = rt4_frame_format_bytes(format);
  const size_t row = static_cast<size_t>(w) * px_bytes;
  for (int32_t i = 0; rc == RT4_OK && i < h; i++)
    if (std::fread(static_cast<unsigned char*>(frame) + static_cast<size_t>(i) * row_stride_px * px_bytes, 1, row, f) != row) {
      rt4_set_err(err, errlen, "%s: truncated checkpoint (row %d of %d)", path, i, h);
      rc = RT4_ERR_PARSE;
    }
  std::fclose(f);
  if (rc != RT4_OK) return rc;
  if (frames_done) *frames_done = hd.frames_done;
  if (seed) *seed = hd.seed;
  return RT4_OK;
}

// ============================================================================ misc
int rt4_abi_version(void) { return RT4_ABI_VERSION; }
size_t rt4_scene_desc_size(void) { return sizeof(rt4_scene_desc); }
size_t rt4_uniforms_size(void) { return sizeof(rt4_uniforms); }

int32_t rt4_frame_format_bytes(int32_t format) {
  switch (format) {
    case RT4_FRAME_RGBA32F: return 16;
    case RT4_FRAME_RGBA16F: return 8;
    case RT4_FRAME_RGBA8: return 4;
    default: return 0;
  }
}

int rt4_progressive_uniforms(const rt4_uniforms* base, uint32_t frame_number, rt4_uniforms* out) {
  if (!base || !out || frame_number == 0) return RT4_ERR_ARG;
  rt4_uniforms u = *base;
  u.part = 1.0f / static_cast<float>(frame_number);  // main.cpp:87 (frameNumber is unsigned, 1.0f / n in fp32)
  u.seed = static_cast<int32_t>(static_cast<uint32_t>(base->seed) ^ (frame_number * 0x9E3779B9u));
  *out = u;
  return RT4_OK;
}

const char* rt4_build_info(void) {
  return "rt4 0.2 " RT4_KERNEL_VERSION " target=gfx950 fp32-contract=off div/sqrt=correctly-rounded built " __DATE__;
}

}  // extern "C"

int rt4_check_render_args(const rt4_uniforms* u, const rt4_region* r, long long row_stride_px, char* err,
                          size_t errlen) {
  if (r->w < 0 || r->h < 0) return rt4_set_err(err, errlen, "negative region size"), RT4_ERR_ARG;
  if (r->w > 0 && row_stride_px < r->w) return rt4_set_err(err, errlen, "row stride smaller than width"), RT4_ERR_ARG;
  if (r->band_rows < 0 || (r->band_rows > 0 && r->band_step < r->band_rows))
    return rt4_set_err(err, errlen, "bad band layout (band_rows %d, band_step %d)", r->band_rows, r->band_step),
           RT4_ERR_ARG;
  // the kernel packs a region-local pixel as j | i << 16 | job << 30 (rt4_trace.hip pack_pixel)
  if (r->w > 65535 || r->h > 16383)
    return rt4_set_err(err, errlen, "region too large (%d x %d; at most 65535 x 16383)", r->w, r->h), RT4_ERR_ARG;
  if (u->samples < 0 || u->reflections_amount < 0)
    return rt4_set_err(err, errlen, "samples/reflections_amount must be >= 0"), RT4_ERR_ARG;
  if (!(u->resolution[0] > 0.0f) || !(u->resolution[1] > 0.0f))
    return rt4_set_err(err, errlen, "resolution must be positive"), RT4_ERR_ARG;
  return RT4_OK;
}

// ============================================================================ scene helpers
namespace {

void set4(float* d, float x, float y, float z, float w) { d[0] = x; d[1] = y; d[2] = z; d[3] = w; }
void copy4(float* d, const float* s) { std::memcpy(d, s, 4 * sizeof(float)); }

rt4_material mat(float glow, float refl, float r, float g, float b) {
  rt4_material m;
  m.glow = glow; m.refl_prob = refl; m.color[0] = r; m.color[1] = g; m.color[2] = b;
  return m;
}

rt4_cylinder make_cylinder(const float* p, const float* a1, const float* a2, float r, const rt4_material& m) {
  rt4_cylinder c;
  copy4(c.point, p); copy4(c.axis1, a1); copy4(c.axis2, a2);
  c.r = r; c.material = m;
  return c;
}

// init_tiger, shader.frag:303-314
rt4_tiger init_tiger(const float* point, const float* a1, const float* a2, const float* a3, const float* a4,
                     float inner_r, float outer_r, const rt4_material& m1, const rt4_material& m2) {
  rt4_tiger t;
  t.inner_cyl1 = make_cylinder(point, a1, a2, inner_r, m1);
  t.outer_cyl1 = make_cylinder(point, a1, a2, outer_r, m1);
  t.inner_cyl2 = make_cylinder(point, a3, a4, inner_r, m2);
  t.outer_cyl2 = make_cylinder(point, a3, a4, outer_r, m2);
  return t;
}

// init_hypercube, shader.frag:374-392: cell k has space(point +/- axis*r, +/-axis) and the other
// three axes. `point + x*r` is a vector multiply-add (one fma per component).
rt4_hypercube init_hypercube(const float* point, const float* x, const float* y, const float* z, const float* w,
                             float r, const rt4_material* m /* 8: xp yp zp wp xn yn zn wn */) {
  const float* ax[4] = {x, y, z, w};
  static const int others[4][3] = {{1, 2, 3}, {0, 2, 3}, {0, 1, 3}, {0, 1, 2}};
  rt4_hypercube h;
  for (int s = 0; s < 2; s++) {
    for (int a = 0; a < 4; a++) {
      rt4_cube& c = h.cubes[s * 4 + a];
      const float sr = s == 0 ? r : -r;
      for (int k = 0; k < 4; k++) {
        c.point[k] = std::fmaf(ax[a][k], sr, point[k]);
        c.norm[k] = s == 0 ? ax[a][k] : -ax[a][k];
      }
      copy4(c.x, ax[others[a][0]]);
      copy4(c.y, ax[others[a][1]]);
      copy4(c.z, ax[others[a][2]]);
      c.r = r;
      c.material = m[s * 4 + a];
    }
  }
  return h;
}

void add_group(rt4_scene_desc& s, int kind, int first, int count, int outer) {
  rt4_group& g = s.groups[s.n_groups++];
  g.kind = kind; g.first = first; g.count = count; g.outer = outer; g.new_first = 1;
}

void std_sun(rt4_scene_desc& s, float sr, float sg, float sb, float lr, float lg, float lb, float sharp) {
  s.sky_light[0] = sr; s.sky_light[1] = sg; s.sky_light[2] = sb;
  set4(s.sun.drct, 0, 1, 1, 0);
  s.sun.angular_size = PI_F * 0.09f;
  s.sun.light[0] = lr; s.sun.light[1] = lg; s.sun.light[2] = lb;
  s.sun.sharpness = sharp;
  s.final_light_mode = RT4_FINAL_LIGHT_SUN_SKY;
}

void ground(rt4_scene_desc& s, const rt4_material& m) {
  rt4_space& sp = s.spaces[s.n_spaces++];
  set4(sp.point, 0, 0, -1.5f, 0);
  set4(sp.norm, 0, 0, 1, 0);
  sp.material = m;
}

}  // namespace

extern "C" int rt4_scene_builtin(const char* name, rt4_scene_desc* out, char* err, size_t errlen) {
  if (!name || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  rt4_scene_desc s;
  std::memset(&s, 0, sizeof s);
  const std::string n(name);
  const float p0[4] = {0, 2, 0, 0};
  const float ex[4] = {1, 0, 0, 0}, ey[4] = {0, 1, 0, 0}, ez[4] = {0, 0, 1, 0}, ew[4] = {0, 0, 0, 1};
  if (n == "sphere") {  // scenes/Шар, плоскость и светилник.frag:3-30
    std_sun(s, 0.02f, 0.06f, 0.12f, 10, 10, 0.95f, 0.8f);
    ground(s, mat(0, 0, 0.6f, 0.4f, 0.2f));
    rt4_sphere& a = s.spheres[s.n_spheres++];
    set4(a.center, -1, 1, 0, 0); a.r = 1.0f; a.material = mat(0, 0.7f, 0.2f, 1.0f, 0.2f);
    rt4_sphere& b = s.spheres[s.n_spheres++];
    set4(b.center, 1, 1, 0, 0); b.r = 0.5f; b.material = mat(90, 0.0f, 1, 1, 1);
    add_group(s, RT4_GROUP_SPACES, 0, s.n_spaces, 0);
    add_group(s, RT4_GROUP_SPHERES, 0, s.n_spheres, 1);
  } else if (n == "room") {  // scenes/Комната со сферой.frag:3-40
    const float size = 3.5f;
    const rt4_material wm[8] = {mat(0, 0, 0.44f, 0.04f, 0.67f), mat(0, 0, 1.0f, 1.0f, 0.0f),
                                mat(0, 0, 1.0f, 0.0f, 0.0f),    mat(0, 0, 0.0f, 0.8f, 0.0f),
                                mat(0, 0, 1.0f, 1.0f, 1.0f),    mat(0, 0, 1.0f, 1.0f, 1.0f),
                                mat(0, 0, 1.0f, 0.67f, 0.0f),   mat(0, 0, 0.07f, 0.25f, 0.67f)};
    const float* axes[4] = {ex, ey, ez, ew};
    for (int k = 0; k < 8; k++) {
      rt4_space& sp = s.spaces[s.n_spaces++];
      const float sz = (k & 1) ? -size : size;
      set4(sp.point, 0, 0, 0, 0);
      sp.point[k / 2] = sz;
      copy4(sp.norm, axes[k / 2]);
      sp.material = wm[k];
    }
    rt4_sphere& a = s.spheres[s.n_spheres++];
    set4(a.center, 0, 0, -size / 5, 0); a.r = 0.35f * size; a.material = mat(0, 0, 1, 1, 1);
    rt4_sphere& b = s.spheres[s.n_spheres++];
    set4(b.center, 0, 0, size, 0); b.r = 0.25f * size; b.material = mat(200, 0, 1, 1, 1);
    add_group(s, RT4_GROUP_SPACES, 0, s.n_spaces, 0);
    add_group(s, RT4_GROUP_SPHERES, 0, s.n_spheres, 1);
    s.final_light_mode = RT4_FINAL_LIGHT_CONSTANT;  // final_light returns vec3(0) (:38-40)
  } else if (n == "tiger") {  // scenes/Фигура tiger.frag:3-30 == executable/shader.frag:414-451
    std_sun(s, 0.2f, 0.6f, 1.2f, 500, 500, 10, 0.0f);
    ground(s, mat(0, 0, 0.4f, 0.25f, 0.07f));
    s.tigers[s.n_tigers++] = init_tiger(p0, ex, ew, ez, ey, 0.9f, 1.4f, mat(0, 0, 1.0f, 0.0f, 0.0f),
                                        mat(0, 0, 0.07f, 0.67f, 0.25f));
    add_group(s, RT4_GROUP_SPACES, 0, s.n_spaces, 0);
    add_group(s, RT4_GROUP_TIGER, 0, 1, 0);
  } else if (n == "cylinder4d") {  // scenes/Четырёхмерный цилиндр.frag:3-38
    std_sun(s, 0.2f, 0.6f, 1.2f, 500, 500, 10, 0.0f);
    ground(s, mat(0, 0, 0.4f, 0.25f, 0.07f));
    rt4_cylinders_union& u = s.unions[s.n_unions++];
    u.cylinder1 = make_cylinder(p0, ex, ew, 1.0f, mat(0, 0, 1.0f, 0.0f, 0.0f));
    u.cylinder2 = make_cylinder(p0, ez, ey, 1.0f, mat(0, 0, 0.07f, 0.67f, 0.25f));
    add_group(s, RT4_GROUP_SPACES, 0, s.n_spaces, 0);
    add_group(s, RT4_GROUP_CYLINDERS_UNION, 0, 1, 1);
  } else if (n == "hypercube") {  // scenes/Гиперкуб.frag:3-37
    std_sun(s, 0.4f, 0.6f, 1.53f, 2100, 1000, 20, 0.0f);
    ground(s, mat(0, 0, 1, 1, 1));
    const rt4_material m[8] = {mat(0, 0, 0.72f, 0.07f, 0.20f), mat(0, 0, 0.00f, 0.61f, 0.28f),
                               mat(0, 0, 1.00f, 0.84f, 0.00f), mat(0, 0, 0.40f, 0.00f, 0.80f),
                               mat(0, 0, 1.00f, 0.35f, 0.00f), mat(0, 0, 0.00f, 0.27f, 0.68f),
                               mat(0, 0, 1.00f, 1.00f, 1.00f), mat(0, 0, 0.01f, 0.01f, 0.01f)};
    s.hypercubes[s.n_hypercubes++] = init_hypercube(p0, ex, ey, ez, ew, 1.0f, m);
    add_group(s, RT4_GROUP_SPACES, 0, s.n_spaces, 0);
    add_group(s, RT4_GROUP_HYPERCUBE, 0, 1, 0);
  } else {
    rt4_set_err(err, errlen, "unknown builtin scene \"%s\" (sphere, room, tiger, cylinder4d, hypercube)", name);
    return RT4_ERR_ARG;
  }
  *out = s;
  return RT4_OK;
}

extern "C" int rt4_scene_validate(const rt4_scene_desc* s, char* err, size_t errlen) {
  if (!s) return rt4_set_err(err, errlen, "NULL scene"), RT4_ERR_ARG;
  if (s->n_groups < 0 || s->n_groups > RT4_MAX_GROUPS || s->n_spaces < 0 || s->n_spaces > RT4_MAX_SPACES ||
      s->n_spheres < 0 || s->n_spheres > RT4_MAX_SPHERES || s->n_cylinders < 0 || s->n_cylinders > RT4_MAX_CYLINDERS ||
      s->n_unions < 0 || s->n_unions > RT4_MAX_UNIONS || s->n_hypercubes < 0 || s->n_hypercubes > RT4_MAX_HYPERCUBES ||
      s->n_tigers < 0 || s->n_tigers > RT4_MAX_TIGERS)
    return rt4_set_err(err, errlen, "scene object counts out of range"), RT4_ERR_CAPACITY;
  if (s->final_light_mode != RT4_FINAL_LIGHT_SUN_SKY && s->final_light_mode != RT4_FINAL_LIGHT_CONSTANT)
    return rt4_set_err(err, errlen, "bad final_light_mode %d", s->final_light_mode), RT4_ERR_ARG;
  for (int g = 0; g < s->n_groups; g++) {
    const rt4_group& gr = s->groups[g];
    int n = 0;
    switch (gr.kind) {
      case RT4_GROUP_SPACES: n = s->n_spaces; break;
      case RT4_GROUP_SPHERES: n = s->n_spheres; break;
      case RT4_GROUP_CYLINDERS: n = s->n_cylinders; break;
      case RT4_GROUP_CYLINDERS_UNION: n = s->n_unions; break;
      case RT4_GROUP_HYPERCUBE: n = s->n_hypercubes; break;
      case RT4_GROUP_TIGER: n = s->n_tigers; break;
      default: return rt4_set_err(err, errlen, "group %d: bad kind %d", g, gr.kind), RT4_ERR_ARG;
    }
    if (gr.first < 0 || gr.count < 0 || gr.first + gr.count > n)
      return rt4_set_err(err, errlen, "group %d: objects [%d, %d) out of range (%d)", g, gr.first, gr.first + gr.count, n),
             RT4_ERR_ARG;
  }
  return RT4_OK;
}

// ============================================================================ GLSL-subset scene loader
namespace {

enum TokKind { T_EOF, T_IDENT, T_NUM, T_PUNCT };
struct Tok {
  TokKind k;
  std::string s;
  int line;
};

bool tokenize(const std::string& src, std::vector<Tok>& out, std::string& msg) {
  size_t i = 0, n = src.size();
  int line = 1;
  bool line_start = true;
  static const char* multi[] = {"<<=", ">>=", "<=", ">=", "==", "!=", "&&", "||", "^^", "++", "--", "+=", "-=",
                                "*=",  "/=",  "%=", "<<", ">>", "&=", "|=", "^="};
  while (i < n) {
    char c = src[i];
    if (c == '\n') { ++line; ++i; line_start = true; continue; }
    if (c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v') { ++i; continue; }
    if (line_start && c == '#') {  // preprocessor line (#version 330)
      while (i < n && src[i] != '\n') ++i;
      continue;
    }
    line_start = false;
    if (c == '/' && i + 1 < n && src[i + 1] == '/') {
      while (i < n && src[i] != '\n') ++i;
      continue;
    }
    if (c == '/' && i + 1 < n && src[i + 1] == '*') {
      i += 2;
      while (i + 1 < n && !(src[i] == '*' && src[i + 1] == '/')) { if (src[i] == '\n') ++line; ++i; }
      if (i + 1 >= n) { msg = "unterminated /* comment"; return false; }
      i += 2;
      continue;
    }
    const unsigned char uc = static_cast<unsigned char>(c);
    if (std::isalpha(uc) || c == '_' || uc >= 0x80) {  // identifiers (UTF-8 bytes allowed)
      size_t b = i;
      while (i < n && (std::isalnum(static_cast<unsigned char>(src[i])) || src[i] == '_' ||
                       static_cast<unsigned char>(src[i]) >= 0x80))
        ++i;
      out.push_back({T_IDENT, src.substr(b, i - b), line});
      continue;
    }
    if (std::isdigit(uc) || (c == '.' && i + 1 < n && std::isdigit(static_cast<unsigned char>(src[i + 1])))) {
      size_t b = i;
      if (c == '0' && i + 1 < n && (src[i + 1] == 'x' || src[i + 1] == 'X')) {
        i += 2;
        while (i < n && std::isxdigit(static_cast<unsigned char>(src[i]))) ++i;
      } else {
        while (i < n && std::isdigit(static_cast<unsigned char>(src[i]))) ++i;
        if (i < n && src[i] == '.') { ++i; while (i < n && std::isdigit(static_cast<unsigned char>(src[i]))) ++i; }
        if (i < n && (src[i] == 'e' || src[i] == 'E')) {
          size_t save = i;
          ++i;
          if (i < n && (src[i] == '+' || src[i] == '-')) ++i;
          if (i < n && std::isdigit(static_cast<unsigned char>(src[i]))) {
            while (i < n && std::isdigit(static_cast<unsigned char>(src[i]))) ++i;
          } else {
            i = save;
          }
        }
      }
      if (i < n && (src[i] == 'f' || src[i] == 'F' || src[i] == 'u' || src[i] == 'U')) ++i;
      else if (i + 1 < n && (src[i] == 'l' || src[i] == 'L') && (src[i + 1] == 'f' || src[i + 1] == 'F')) i += 2;
      out.push_back({T_NUM, src.substr(b, i - b), line});
      continue;
    }
    bool matched = false;
    for (const char* m : multi) {
      size_t L = std::strlen(m);
      if (src.compare(i, L, m) == 0) {
        out.push_back({T_PUNCT, m, line});
        i += L;
        matched = true;
        break;
      }
    }
    if (matched) continue;
    out.push_back({T_PUNCT, std::string(1, c), line});
    ++i;
  }
  out.push_back({T_EOF, "", line});
  return true;
}

// ---- values of the constant-expression evaluator
struct Val {
  enum K { NONE, NUM, BOOL, VEC, STRUCT, ARRAY } k = NONE;
  bool isint = false;
  float f = 0.0f;
  long long i = 0;
  bool b = false;
  std::vector<float> v;    // VEC
  std::string type;        // STRUCT: struct name; ARRAY: element type
  std::vector<Val> items;  // STRUCT fields / ARRAY elements
};

Val num_f(float f) { Val r; r.k = Val::NUM; r.f = f; return r; }
Val num_i(long long i) { Val r; r.k = Val::NUM; r.isint = true; r.i = i; r.f = static_cast<float>(i); return r; }
Val vecv(std::vector<float> v) { Val r; r.k = Val::VEC; r.v = std::move(v); return r; }
Val strct(const std::string& t, std::vector<Val> items) { Val r; r.k = Val::STRUCT; r.type = t; r.items = std::move(items); return r; }

struct StructSpec { const char* name; std::vector<std::string> fields; std::vector<std::string> types; };
// Field lists of the scene structs (shader.frag:32-35, 163-167, 189-192, 225-228, 243-247, 279-281,
// 298-300, 345-350, 370-372, 404-409). type: "float", "vec3", "vec4", or a struct name / "visible_cube[8]".
const std::vector<StructSpec>& struct_specs() {
  static const std::vector<StructSpec> specs = {
      {"material", {"glow", "refl_prob", "color"}, {"float", "float", "vec3"}},
      {"space", {"point", "norm"}, {"vec4", "vec4"}},
      {"sphere", {"center", "r"}, {"vec4", "float"}},
      {"line", {"point", "drct"}, {"vec4", "vec4"}},
      {"ray", {"point", "drct"}, {"vec4", "vec4"}},
      {"visible_space", {"figure", "material"}, {"space", "material"}},
      {"visible_sphere", {"figure", "material"}, {"sphere", "material"}},
      {"visible_cylinder", {"point", "axis1", "axis2", "r", "material"}, {"vec4", "vec4", "vec4", "float", "material"}},
      {"visible_cylinders_union", {"cylinder1", "cylinder2"}, {"visible_cylinder", "visible_cylinder"}},
      {"visible_tiger",
       {"inner_cyl1", "outer_cyl1", "inner_cyl2", "outer_cyl2"},
       {"visible_cylinder", "visible_cylinder", "visible_cylinder", "visible_cylinder"}},
      {"visible_cube", {"space", "x", "y", "z", "r", "material"}, {"space", "vec4", "vec4", "vec4", "float", "material"}},
      {"visible_hypercube", {"cubes"}, {"visible_cube[8]"}},
      {"sun_properties", {"drct", "angular_size", "light", "sharpness"}, {"vec4", "float", "vec3", "float"}},
  };
  return specs;
}
const StructSpec* find_spec(const std::string& n) {
  for (const auto& s : struct_specs())
    if (n == s.name) return &s;
  return nullptr;
}

struct ParseError {
  std::string msg;
};

[[noreturn]] void fail(const Tok& t, const std::string& m) {
  throw ParseError{"line " + std::to_string(t.line) + ": " + m + (t.k == T_EOF ? " (at end of input)" : " (at '" + t.s + "')")};
}

bool is_vec_type(const std::string& t, int& n) {
  if (t == "vec2") { n = 2; return true; }
  if (t == "vec3") { n = 3; return true; }
  if (t == "vec4") { n = 4; return true; }
  return false;
}

// Converts v to the declared field/parameter type, with GLSL 330 implicit int->float conversion.
Val coerce(const Val& v, const std::string& type, const Tok& at) {
  int n;
  if (type == "float") {
    if (v.k != Val::NUM) fail(at, "expected a scalar for a float");
    return num_f(v.isint ? static_cast<float>(v.i) : v.f);
  }
  if (type == "int" || type == "uint") {
    if (v.k != Val::NUM || !v.isint) fail(at, "expected an integer");
    return v;
  }
  if (type == "bool") {
    if (v.k != Val::BOOL) fail(at, "expected a bool");
    return v;
  }
  if (is_vec_type(type, n)) {
    if (v.k != Val::VEC || static_cast<int>(v.v.size()) != n) fail(at, "expected " + type);
    return v;
  }
  if (type == "visible_cube[8]") {
    if (v.k != Val::ARRAY || v.type != "visible_cube" || v.items.size() != 8) fail(at, "expected visible_cube[8]");
    return v;
  }
  if (v.k != Val::STRUCT || v.type != type) fail(at, "expected " + type);
  return v;
}

class Evaluator {
 public:
  Evaluator(const std::vector<Tok>& t, std::map<std::string, Val>& sym) : t_(t), sym_(sym) {}

  Val eval_range(size_t b, size_t e) {
    p_ = b;
    end_ = e;
    Val v = additive();
    if (p_ != end_) fail(t_[p_], "unexpected token in expression");
    return v;
  }

 private:
  const std::vector<Tok>& t_;
  std::map<std::string, Val>& sym_;
  size_t p_ = 0, end_ = 0;

  const Tok& cur() const { return p_ < end_ ? t_[p_] : t_.back(); }
  bool at(const char* s) const { return p_ < end_ && t_[p_].k == T_PUNCT && t_[p_].s == s; }
  void expect(const char* s) {
    if (!at(s)) fail(cur(), std::string("expected '") + s + "'");
    ++p_;
  }

  static Val arith(char op, const Val& a, const Val& b, const Tok& at) {
    if (a.k == Val::NUM && b.k == Val::NUM) {
      if (a.isint && b.isint) {
        switch (op) {
          case '+': return num_i(a.i + b.i);
          case '-': return num_i(a.i - b.i);
          case '*': return num_i(a.i * b.i);
          default:
            if (b.i == 0) fail(at, "integer division by zero");
            return num_i(a.i / b.i);
        }
      }
      const float x = a.isint ? static_cast<float>(a.i) : a.f, y = b.isint ? static_cast<float>(b.i) : b.f;
      switch (op) {
        case '+': return num_f(x + y);
        case '-': return num_f(x - y);
        case '*': return num_f(x * y);
        default: return num_f(x / y);
      }
    }
    auto comp = [&](float x, float y) {
      switch (op) {
        case '+': return x + y;
        case '-': return x - y;
        case '*': return x * y;
        default: return x / y;
      }
    };
    auto sc = [](const Val& v) { return v.isint ? static_cast<float>(v.i) : v.f; };
    if (a.k == Val::VEC && b.k == Val::VEC) {
      if (a.v.size() != b.v.size()) fail(at, "vector size mismatch");
      std::vector<float> r(a.v.size());
      for (size_t k = 0; k < r.size(); k++) r[k] = comp(a.v[k], b.v[k]);
      return vecv(r);
    }
    if (a.k == Val::VEC && b.k == Val::NUM) {
      std::vector<float> r(a.v.size());
      for (size_t k = 0; k < r.size(); k++) r[k] = comp(a.v[k], sc(b));
      return vecv(r);
    }
    if (a.k == Val::NUM && b.k == Val::VEC) {
      std::vector<float> r(b.v.size());
      for (size_t k = 0; k < r.size(); k++) r[k] = comp(sc(a), b.v[k]);
      return vecv(r);
    }
    fail(at, "unsupported operands of arithmetic");
  }

  Val additive() {
    Val v = multiplicative();
    while (at("+") || at("-")) {
      const Tok& op = cur();
      ++p_;
      Val r = multiplicative();
      v = arith(op.s[0], v, r, op);
    }
    return v;
  }
  Val multiplicative() {
    Val v = unary();
    while (at("*") || at("/")) {
      const Tok& op = cur();
      ++p_;
      Val r = unary();
      v = arith(op.s[0], v, r, op);
    }
    return v;
  }
  Val unary() {
    if (at("-")) {
      const Tok& op = cur();
      ++p_;
      Val v = unary();
      if (v.k == Val::NUM) return v.isint ? num_i(-v.i) : num_f(-v.f);
      if (v.k == Val::VEC) {
        for (auto& x : v.v) x = -x;
        return v;
      }
      fail(op, "cannot negate this value");
    }
    if (at("+")) { ++p_; return unary(); }
    return postfix();
  }
  Val postfix() {
    Val v = primary();
    while (true) {
      if (at(".")) {
        ++p_;
        const Tok& f = cur();
        if (f.k != T_IDENT) fail(f, "expected a field name");
        ++p_;
        v = member(v, f);
      } else if (at("[")) {
        const Tok& b = cur();
        ++p_;
        Val idx = additive();
        expect("]");
        if (idx.k != Val::NUM || !idx.isint) fail(b, "array index must be an integer constant");
        if (v.k == Val::ARRAY) {
          if (idx.i < 0 || idx.i >= static_cast<long long>(v.items.size())) fail(b, "index out of range");
          v = Val(v.items[static_cast<size_t>(idx.i)]);
        } else if (v.k == Val::VEC) {
          if (idx.i < 0 || idx.i >= static_cast<long long>(v.v.size())) fail(b, "index out of range");
          v = num_f(v.v[static_cast<size_t>(idx.i)]);
        } else {
          fail(b, "indexing a non-array");
        }
      } else {
        return v;
      }
    }
  }
  static Val member(const Val& v, const Tok& f) {
    if (v.k == Val::VEC) {
      static const std::string sets[3] = {"xyzw", "rgba", "stpq"};
      std::vector<float> r;
      for (char c : f.s) {
        int idx = -1;
        for (const auto& s : sets) {
          auto pos = s.find(c);
          if (pos != std::string::npos) idx = static_cast<int>(pos);
        }
        if (idx < 0 || idx >= static_cast<int>(v.v.size())) fail(f, "bad swizzle");
        r.push_back(v.v[static_cast<size_t>(idx)]);
      }
      if (r.size() == 1) return num_f(r[0]);
      return vecv(r);
    }
    if (v.k == Val::STRUCT) {
      const StructSpec* sp = find_spec(v.type);
      for (size_t k = 0; sp && k < sp->fields.size(); k++)
        if (sp->fields[k] == f.s) return v.items[k];
      fail(f, "no field '" + f.s + "' in " + v.type);
    }
    if (v.k == Val::ARRAY && f.s == "length") return v;  // handled by call syntax `.length()` below
    fail(f, "member access on a non-struct");
  }

  std::vector<Val> args() {
    std::vector<Val> a;
    expect("(");
    if (at(")")) { ++p_; return a; }
    while (true) {
      a.push_back(additive());
      if (at(",")) { ++p_; continue; }
      expect(")");
      return a;
    }
  }

  Val construct(const Tok& name, std::vector<Val> a) {
    const std::string& n = name.s;
    int vn;
    if (is_vec_type(n, vn)) {  // vecN(...): scalars and vectors flattened; one scalar splats
      std::vector<float> comps;
      for (const auto& x : a) {
        if (x.k == Val::NUM) comps.push_back(x.isint ? static_cast<float>(x.i) : x.f);
        else if (x.k == Val::VEC) comps.insert(comps.end(), x.v.begin(), x.v.end());
        else fail(name, n + "(): bad argument");
      }
      if (a.size() == 1 && a[0].k == Val::NUM) return vecv(std::vector<float>(static_cast<size_t>(vn), comps[0]));
      // GLSL: enough components, and the last argument must contribute at least one of them
      const size_t last = a.empty() ? 0 : (a.back().k == Val::VEC ? a.back().v.size() : 1);
      if (comps.size() < static_cast<size_t>(vn) || comps.size() - last >= static_cast<size_t>(vn))
        fail(name, n + "(): wrong number of components");
      comps.resize(static_cast<size_t>(vn));
      return vecv(comps);
    }
    if (n == "float" || n == "int" || n == "uint") {
      if (a.size() != 1 || a[0].k != Val::NUM) fail(name, n + "(): expects one scalar");
      if (n == "float") return num_f(a[0].isint ? static_cast<float>(a[0].i) : a[0].f);
      return num_i(a[0].isint ? a[0].i : static_cast<long long>(a[0].f));
    }
    if (n == "init_tiger") {  // shader.frag:303-314
      if (a.size() != 9) fail(name, "init_tiger expects 9 arguments");
      std::vector<Val> c;
      const std::string ts[9] = {"vec4", "vec4", "vec4", "vec4", "vec4", "float", "float", "material", "material"};
      for (int k = 0; k < 9; k++) a[static_cast<size_t>(k)] = coerce(a[static_cast<size_t>(k)], ts[k], name);
      auto cyl = [&](const Val& ax1, const Val& ax2, const Val& r, const Val& m) {
        return strct("visible_cylinder", {a[0], ax1, ax2, r, m});
      };
      return strct("visible_tiger", {cyl(a[1], a[2], a[5], a[7]), cyl(a[1], a[2], a[6], a[7]),
                                     cyl(a[3], a[4], a[5], a[8]), cyl(a[3], a[4], a[6], a[8])});
    }
    if (n == "init_hypercube") {  // shader.frag:374-392
      if (a.size() != 14) fail(name, "init_hypercube expects 14 arguments");
      for (int k = 0; k < 5; k++) a[static_cast<size_t>(k)] = coerce(a[static_cast<size_t>(k)], "vec4", name);
      a[5] = coerce(a[5], "float", name);
      for (int k = 6; k < 14; k++) a[static_cast<size_t>(k)] = coerce(a[static_cast<size_t>(k)], "material", name);
      const float r = a[5].f;
      static const int others[4][3] = {{2, 3, 4}, {1, 3, 4}, {1, 2, 4}, {1, 2, 3}};
      Val arr;
      arr.k = Val::ARRAY;
      arr.type = "visible_cube";
      for (int s = 0; s < 2; s++) {
        for (int ax = 0; ax < 4; ax++) {
          const Val& axis = a[static_cast<size_t>(1 + ax)];
          std::vector<float> pt(4), nm(4);
          for (int k = 0; k < 4; k++) {
            pt[static_cast<size_t>(k)] = std::fmaf(axis.v[static_cast<size_t>(k)], s == 0 ? r : -r, a[0].v[static_cast<size_t>(k)]);
            nm[static_cast<size_t>(k)] = s == 0 ? axis.v[static_cast<size_t>(k)] : -axis.v[static_cast<size_t>(k)];
          }
          arr.items.push_back(strct("visible_cube", {strct("space", {vecv(pt), vecv(nm)}), a[static_cast<size_t>(others[ax][0])],
                                                     a[static_cast<size_t>(others[ax][1])], a[static_cast<size_t>(others[ax][2])],
                                                     a[5], a[static_cast<size_t>(6 + s * 4 + ax)]}));
        }
      }
      return strct("visible_hypercube", {arr});
    }
    const StructSpec* sp = find_spec(n);
    if (!sp) fail(name, "unknown function or constructor '" + n + "'");
    if (a.size() != sp->fields.size()) fail(name, n + "(): expects " + std::to_string(sp->fields.size()) + " arguments");
    for (size_t k = 0; k < a.size(); k++) a[k] = coerce(a[k], sp->types[k], name);
    return strct(n, a);
  }

  Val primary() {
    const Tok& t = cur();
    if (at("(")) {
      ++p_;
      Val v = additive();
      expect(")");
      return v;
    }
    if (t.k == T_NUM) {
      ++p_;
      const std::string& s = t.s;
      const bool hex = s.size() > 1 && (s[1] == 'x' || s[1] == 'X');
      const bool isfloat = !hex && (s.find_first_of(".eEfF") != std::string::npos);
      if (isfloat) {
        std::string body = s;
        while (!body.empty() && (body.back() == 'f' || body.back() == 'F' || body.back() == 'l' || body.back() == 'L'))
          body.pop_back();
        return num_f(std::strtof(body.c_str(), nullptr));  // GLSL float literal: nearest fp32
      }
      return num_i(std::strtoll(s.c_str(), nullptr, 0));
    }
    if (t.k == T_IDENT) {
      ++p_;
      if (t.s == "true" || t.s == "false") {
        Val v;
        v.k = Val::BOOL;
        v.b = t.s == "true";
        return v;
      }
      if (at("[") && (find_spec(t.s) != nullptr)) {  // array constructor T[N](...) / T[](...)
        const Tok& b = cur();
        ++p_;
        long long want = -1;
        if (!at("]")) {
          Val nv = additive();
          if (nv.k != Val::NUM || !nv.isint) fail(b, "array size must be an integer constant");
          want = nv.i;
        }
        expect("]");
        std::vector<Val> a = args();
        if (want >= 0 && want != static_cast<long long>(a.size())) fail(b, "array constructor size mismatch");
        Val arr;
        arr.k = Val::ARRAY;
        arr.type = t.s;
        for (auto& x : a) arr.items.push_back(coerce(x, t.s, b));
        return arr;
      }
      if (at("(")) return construct(t, args());
      auto it = sym_.find(t.s);
      if (it == sym_.end()) fail(t, "unknown identifier '" + t.s + "'");
      Val v = it->second;
      if (at(".") && p_ + 2 < end_ && t_[p_ + 1].s == "length" && t_[p_ + 2].s == "(") {  // arr.length()
        if (v.k != Val::ARRAY) fail(t, "length() of a non-array");
        p_ += 3;
        expect(")");
        return num_i(static_cast<long long>(v.items.size()));
      }
      return v;
    }
    fail(t, "expected an expression");
  }
};

// ---- Val -> rt4_* conversion
void put4(float* d, const Val& v) { for (int k = 0; k < 4; k++) d[k] = v.v[static_cast<size_t>(k)]; }
rt4_material to_mat(const Val& m) {
  rt4_material r;
  r.glow = m.items[0].f;
  r.refl_prob = m.items[1].f;
  for (int k = 0; k < 3; k++) r.color[k] = m.items[2].v[static_cast<size_t>(k)];
  return r;
}
rt4_cylinder to_cyl(const Val& c) {
  rt4_cylinder r;
  put4(r.point, c.items[0]); put4(r.axis1, c.items[1]); put4(r.axis2, c.items[2]);
  r.r = c.items[3].f;
  r.material = to_mat(c.items[4]);
  return r;
}

struct Decl {
  std::string type;  // declared type (array types as "T[]")
  Val value;
  bool ok = false;
  std::string error;
};

struct Func {
  size_t body_b = 0, body_e = 0;  // token range inside { }
  bool present = false;
};

size_t match_close(const std::vector<Tok>& t, size_t open) {  // index of the token closing t[open]
  const std::string o = t[open].s, c = o == "(" ? ")" : o == "[" ? "]" : "}";
  int depth = 0;
  for (size_t i = open; i < t.size(); i++) {
    if (t[i].k == T_PUNCT && t[i].s == o) ++depth;
    else if (t[i].k == T_PUNCT && t[i].s == c && --depth == 0) return i;
    if (t[i].k == T_EOF) break;
  }
  fail(t[open], "unbalanced '" + o + "'");
}

struct SceneBuild {
  rt4_scene_desc d;
  std::map<std::string, std::pair<int, int>> placed;  // variable -> (first, count) in its kind's array
};

int place_objects(SceneBuild& sb, const std::string& var, const Decl& decl, int kind, const Tok& at) {
  auto it = sb.placed.find(var);
  if (it != sb.placed.end()) return it->second.first;
  const Val& v = decl.value;
  std::vector<const Val*> objs;
  if (v.k == Val::ARRAY) for (const auto& x : v.items) objs.push_back(&x);
  else objs.push_back(&v);
  rt4_scene_desc& d = sb.d;
  int first = 0;
  auto need = [&](int have, int add, int cap) {
    if (have + add > cap) fail(at, "too many objects of this kind (limit " + std::to_string(cap) + ")");
  };
  const int cnt = static_cast<int>(objs.size());
  switch (kind) {
    case RT4_GROUP_SPACES:
      need(d.n_spaces, cnt, RT4_MAX_SPACES);
      first = d.n_spaces;
      for (const Val* o : objs) {
        if (o->type != "visible_space") fail(at, "space_intersection needs visible_space objects");
        rt4_space& s = d.spaces[d.n_spaces++];
        put4(s.point, o->items[0].items[0]);
        put4(s.norm, o->items[0].items[1]);
        s.material = to_mat(o->items[1]);
      }
      break;
    case RT4_GROUP_SPHERES:
      need(d.n_spheres, cnt, RT4_MAX_SPHERES);
      first = d.n_spheres;
      for (const Val* o : objs) {
        if (o->type != "visible_sphere") fail(at, "sphere_intersection needs visible_sphere objects");
        rt4_sphere& s = d.spheres[d.n_spheres++];
        put4(s.center, o->items[0].items[0]);
        s.r = o->items[0].items[1].f;
        s.material = to_mat(o->items[1]);
      }
      break;
    case RT4_GROUP_CYLINDERS:
      need(d.n_cylinders, cnt, RT4_MAX_CYLINDERS);
      first = d.n_cylinders;
      for (const Val* o : objs) {
        if (o->type != "visible_cylinder") fail(at, "cylinder_intersection needs visible_cylinder objects");
        d.cylinders[d.n_cylinders++] = to_cyl(*o);
      }
      break;
    case RT4_GROUP_CYLINDERS_UNION:
      need(d.n_unions, cnt, RT4_MAX_UNIONS);
      first = d.n_unions;
      for (const Val* o : objs) {
        if (o->type != "visible_cylinders_union") fail(at, "cylinders_union_intersection needs visible_cylinders_union");
        rt4_cylinders_union& u = d.unions[d.n_unions++];
        u.cylinder1 = to_cyl(o->items[0]);
        u.cylinder2 = to_cyl(o->items[1]);
      }
      break;
    case RT4_GROUP_HYPERCUBE:
      need(d.n_hypercubes, cnt, RT4_MAX_HYPERCUBES);
      first = d.n_hypercubes;
      for (const Val* o : objs) {
        if (o->type != "visible_hypercube") fail(at, "hypercube_intersection needs visible_hypercube");
        rt4_hypercube& h = d.hypercubes[d.n_hypercubes++];
        for (int k = 0; k < 8; k++) {
          const Val& c = o->items[0].items[static_cast<size_t>(k)];
          rt4_cube& cb = h.cubes[k];
          put4(cb.point, c.items[0].items[0]);
          put4(cb.norm, c.items[0].items[1]);
          put4(cb.x, c.items[1]); put4(cb.y, c.items[2]); put4(cb.z, c.items[3]);
          cb.r = c.items[4].f;
          cb.material = to_mat(c.items[5]);
        }
      }
      break;
    case RT4_GROUP_TIGER:
      need(d.n_tigers, cnt, RT4_MAX_TIGERS);
      first = d.n_tigers;
      for (const Val* o : objs) {
        if (o->type != "visible_tiger") fail(at, "tiger_intersection needs visible_tiger");
        rt4_tiger& t = d.tigers[d.n_tigers++];
        t.inner_cyl1 = to_cyl(o->items[0]);
        t.outer_cyl1 = to_cyl(o->items[1]);
        t.inner_cyl2 = to_cyl(o->items[2]);
        t.outer_cyl2 = to_cyl(o->items[3]);
      }
      break;
    default: fail(at, "internal: bad kind");
  }
  sb.placed[var] = {first, cnt};
  return first;
}

// Parses find_intersection's body (shader.frag:434-451): every `X = closest(A, B);` where one side is
// the accumulator X and the other a `<kind>_intersection(obj, ray[, outer])` call becomes a group.
void parse_find_intersection(const std::vector<Tok>& t, size_t b, size_t e, std::map<std::string, Decl>& decls,
                             std::map<std::string, Val>& sym, SceneBuild& sb) {
  struct KindName { const char* fn; int kind; bool has_outer; };
  static const KindName kinds[] = {{"space_intersection", RT4_GROUP_SPACES, false},
                                   {"sphere_intersection", RT4_GROUP_SPHERES, true},
                                   {"cylinder_intersection", RT4_GROUP_CYLINDERS, true},
                                   {"cylinders_union_intersection", RT4_GROUP_CYLINDERS_UNION, false},
                                   {"hypercube_intersection", RT4_GROUP_HYPERCUBE, false},
                                   {"tiger_intersection", RT4_GROUP_TIGER, false}};
  // loop bound of the innermost enclosing `for (...; i < BOUND; ...)`, if any
  std::vector<std::pair<size_t, long long>> loops;  // (end token of loop body, bound)
  for (size_t i = b; i < e; i++) {
    while (!loops.empty() && i > loops.back().first) loops.pop_back();
    if (t[i].k == T_IDENT && t[i].s == "for") {
      size_t po = i + 1;
      if (t[po].s != "(") fail(t[i], "expected '(' after for");
      size_t pc = match_close(t, po);
      long long bound = -1;
      for (size_t k = po; k < pc; k++) {
        if (t[k].s == "<" || t[k].s == "<=") {
          size_t s2 = k + 1, e2 = s2;
          while (e2 < pc && t[e2].s != ";") ++e2;
          Evaluator ev(t, sym);
          Val bv = ev.eval_range(s2, e2);
          if (bv.k != Val::NUM || !bv.isint) fail(t[k], "for-loop bound must be an integer constant");
          bound = bv.i + (t[k].s == "<=" ? 1 : 0);
          break;
        }
      }
      size_t body_end;
      if (t[pc + 1].s == "{") body_end = match_close(t, pc + 1);
      else { body_end = pc + 1; while (body_end < e && t[body_end].s != ";") ++body_end; }
      loops.push_back({body_end, bound});
      i = pc;
      continue;
    }
    if (!(t[i].k == T_IDENT && t[i].s == "closest" && i >= 2 && t[i - 1].s == "=" && t[i + 1].s == "(")) continue;
    const std::string acc = t[i - 2].s;
    const size_t po = i + 1, pc = match_close(t, po);
    // split the two top-level arguments
    size_t comma = 0;
    int depth = 0;
    for (size_t k = po + 1; k < pc; k++) {
      if (t[k].s == "(" || t[k].s == "[") ++depth;
      else if (t[k].s == ")" || t[k].s == "]") --depth;
      else if (depth == 0 && t[k].s == ",") { comma = k; break; }
    }
    if (!comma) fail(t[i], "closest() needs two arguments");
    const bool first_is_acc = (comma == po + 2 && t[po + 1].s == acc);
    const bool second_is_acc = (pc == comma + 2 && t[comma + 1].s == acc);
    if (first_is_acc == second_is_acc) fail(t[i], "unsupported closest() statement (one argument must be '" + acc + "')");
    const size_t cb = first_is_acc ? comma + 1 : po + 1;  // call tokens [cb, ce)
    const size_t ce = first_is_acc ? pc : comma;
    const KindName* kn = nullptr;
    for (const auto& k : kinds)
      if (t[cb].s == k.fn) kn = &k;
    if (!kn || t[cb + 1].s != "(") fail(t[cb], "unsupported intersection call");
    const size_t cpc = match_close(t, cb + 1);
    if (cpc + 1 != ce) fail(t[cb], "unexpected tokens after the intersection call");
    // first call argument: NAME, NAME[i] or NAME[INT]
    const Tok& objtok = t[cb + 2];
    if (objtok.k != T_IDENT) fail(objtok, "expected an object name");
    auto dit = decls.find(objtok.s);
    if (dit == decls.end() || !dit->second.ok)
      fail(objtok, "object '" + objtok.s + "' is not a defined scene object" +
                       (dit != decls.end() ? " (" + dit->second.error + ")" : std::string()));
    const Decl& decl = dit->second;
    size_t after = cb + 3;
    int sel_first = 0, sel_count = 1;
    const bool is_array = decl.value.k == Val::ARRAY;
    if (t[after].s == "[") {
      size_t cl = match_close(t, after);
      if (!is_array) fail(objtok, "indexing a non-array object");
      const long long len = static_cast<long long>(decl.value.items.size());
      if (cl == after + 2 && t[after + 1].k == T_NUM) {
        long long idx = std::strtoll(t[after + 1].s.c_str(), nullptr, 0);
        if (idx < 0 || idx >= len) fail(t[after + 1], "index out of range");
        sel_first = static_cast<int>(idx);
        sel_count = 1;
      } else {
        if (loops.empty() || loops.back().second < 0) fail(objtok, "array element indexed outside a counted for-loop");
        const long long bound = loops.back().second;
        if (bound > len) fail(objtok, "for-loop bound exceeds the array length");
        sel_first = 0;
        sel_count = static_cast<int>(bound);
      }
      after = cl + 1;
    } else if (is_array) {
      fail(objtok, "array object passed without an index");
    }
    int outer = 1;
    if (kn->has_outer) {
      // remaining args: ray , outer
      size_t k = after;
      if (t[k].s != ",") fail(t[k], "expected ', ray'");
      k += 2;  // skip ray
      if (t[k].s != ",") fail(t[k], kn->fn + std::string(" needs the outer flag"));
      const Tok& ot = t[k + 1];
      if (ot.s == "true") outer = 1;
      else if (ot.s == "false") outer = 0;
      else fail(ot, "outer flag must be true or false");
    }
    const int base = place_objects(sb, objtok.s, decl, kn->kind, objtok);
    if (sb.d.n_groups >= RT4_MAX_GROUPS) fail(t[i], "too many intersection statements");
    rt4_group& g = sb.d.groups[sb.d.n_groups++];
    g.kind = kn->kind;
    g.first = base + sel_first;
    g.count = sel_count;
    g.outer = kn->has_outer ? outer : (kn->kind == RT4_GROUP_CYLINDERS_UNION ? 1 : 0);
    g.new_first = second_is_acc ? 1 : 0;
    i = pc;
  }
}

int parse_scene(const std::string& src, rt4_scene_desc* out, char* err, size_t errlen) {
  std::vector<Tok> t;
  std::string msg;
  if (!tokenize(src, t, msg)) return rt4_set_err(err, errlen, "scene: %s", msg.c_str()), RT4_ERR_PARSE;
  try {
    std::map<std::string, Val> sym;
    sym["PI"] = num_f(PI_F);          // shader.frag:23 (a pasted scene sees these)
    sym["SMALL_FLOAT"] = num_f(SMALL_F);
    std::map<std::string, Decl> decls;
    Func find_fn, final_fn;
    static const char* kScene[] = {"visible_space", "visible_sphere", "visible_cylinder", "visible_cylinders_union",
                                   "visible_tiger", "visible_hypercube", "sun_properties"};
    auto scene_type = [&](const std::string& ty) {
      for (const char* s : kScene)
        if (ty == s) return true;
      return false;
    };
    size_t i = 0;
    while (t[i].k != T_EOF) {
      if (t[i].k == T_PUNCT && t[i].s == ";") { ++i; continue; }
      if (t[i].k != T_IDENT) fail(t[i], "unexpected token at top level");
      if (t[i].s == "struct") {  // struct X { ... } ;
        size_t k = i;
        while (t[k].s != "{" && t[k].k != T_EOF) ++k;
        if (t[k].k == T_EOF) fail(t[i], "bad struct");
        i = match_close(t, k) + 1;
        continue;
      }
      // declaration: qualifiers, type [array], name [array], then ( ... ) | = init | ;
      size_t k = i;
      while (t[k].k == T_IDENT && (t[k].s == "const" || t[k].s == "uniform" || t[k].s == "in" || t[k].s == "out" ||
                                   t[k].s == "highp" || t[k].s == "mediump" || t[k].s == "lowp" || t[k].s == "precision" ||
                                   t[k].s == "flat" || t[k].s == "smooth"))
        ++k;
      const bool is_uniform = [&] { for (size_t q = i; q < k; q++) if (t[q].s == "uniform" || t[q].s == "precision") return true; return false; }();
      if (t[k].k != T_IDENT) fail(t[k], "expected a type");
      std::string type = t[k].s;
      ++k;
      bool arr = false;
      if (t[k].s == "[") { arr = true; k = match_close(t, k) + 1; }
      if (is_uniform) {  // uniform / precision statements: skip
        while (t[k].s != ";" && t[k].k != T_EOF) ++k;
        i = k + 1;
        continue;
      }
      while (true) {
        if (t[k].k != T_IDENT) fail(t[k], "expected a name");
        const Tok& name = t[k];
        ++k;
        bool arr2 = arr;
        if (t[k].s == "[") { arr2 = true; k = match_close(t, k) + 1; }
        if (t[k].s == "(") {  // function definition or prototype
          size_t pc = match_close(t, k);
          if (t[pc + 1].s == "{") {
            size_t bc = match_close(t, pc + 1);
            if (name.s == "find_intersection") find_fn = {pc + 2, bc, true};
            if (name.s == "final_light") final_fn = {pc + 2, bc, true};
            k = bc + 1;
          } else {
            k = pc + 1;
          }
          break;
        }
        Decl d;
        d.type = arr2 ? type + "[]" : type;
        if (t[k].s == "=") {
          size_t s2 = ++k;
          int depth = 0;
          while (t[k].k != T_EOF) {
            if (t[k].s == "(" || t[k].s == "[" || t[k].s == "{") ++depth;
            else if (t[k].s == ")" || t[k].s == "]" || t[k].s == "}") --depth;
            else if (depth == 0 && (t[k].s == ";" || t[k].s == ",")) break;
            ++k;
          }
          try {
            Evaluator ev(t, sym);
            d.value = ev.eval_range(s2, k);
            d.ok = true;
            sym[name.s] = d.value;
          } catch (const ParseError& pe) {
            d.error = pe.msg;
            if (scene_type(type) || name.s == "sky_light") throw;  // a scene object must evaluate
            sym.erase(name.s);
          }
        }
        decls[name.s] = d;
        if (t[k].s == ",") { ++k; continue; }
        if (t[k].s != ";") fail(t[k], "expected ';'");
        ++k;
        break;
      }
      i = k;
    }

    SceneBuild sb;
    std::memset(&sb.d, 0, sizeof sb.d);
    if (!find_fn.present) throw ParseError{"the scene defines no find_intersection(ray) function"};
    parse_find_intersection(t, find_fn.body_b, find_fn.body_e, decls, sym, sb);
    if (sb.d.n_groups == 0) throw ParseError{"find_intersection tests no objects"};

    bool const_light = false;
    if (final_fn.present) {  // `return <constant vec3>;` is a constant override (S-room :38-40)
      const size_t b = final_fn.body_b, e = final_fn.body_e;
      if (t[b].s == "return" && e >= b + 2 && t[e - 1].s == ";") {
        try {
          Evaluator ev(t, sym);
          Val v = ev.eval_range(b + 1, e - 1);
          if (v.k == Val::VEC && v.v.size() == 3) {
            const_light = true;
            sb.d.final_light_mode = RT4_FINAL_LIGHT_CONSTANT;
            for (int q = 0; q < 3; q++) sb.d.final_light_const[q] = v.v[static_cast<size_t>(q)];
          }
        } catch (const ParseError&) {
        }
      }
      if (!const_light) {
        bool uses_sun = false;
        for (size_t q = b; q < e; q++)
          if (t[q].s == "sun") uses_sun = true;
        if (!uses_sun) throw ParseError{"unsupported final_light body (only the default sun/sky model or `return vec3(...)`)"};
      }
    }
    if (!const_light) {
      sb.d.final_light_mode = RT4_FINAL_LIGHT_SUN_SKY;
      auto sk = sym.find("sky_light");
      auto sn = sym.find("sun");
      if (sk == sym.end() || sk->second.k != Val::VEC || sk->second.v.size() != 3)
        throw ParseError{"the scene defines no vec3 sky_light (needed by the default final_light)"};
      if (sn == sym.end() || sn->second.k != Val::STRUCT || sn->second.type != "sun_properties")
        throw ParseError{"the scene defines no sun_properties sun (needed by the default final_light)"};
      for (int q = 0; q < 3; q++) sb.d.sky_light[q] = sk->second.v[static_cast<size_t>(q)];
      const Val& s = sn->second;
      put4(sb.d.sun.drct, s.items[0]);
      sb.d.sun.angular_size = s.items[1].f;
      for (int q = 0; q < 3; q++) sb.d.sun.light[q] = s.items[2].v[static_cast<size_t>(q)];
      sb.d.sun.sharpness = s.items[3].f;
    }
    int st = rt4_scene_validate(&sb.d, err, errlen);
    if (st != RT4_OK) return st;
    *out = sb.d;
    return RT4_OK;
  } catch (const ParseError& pe) {
    rt4_set_err(err, errlen, "scene: %s", pe.msg.c_str());
    return RT4_ERR_PARSE;
  }
}

}  // namespace

extern "C" int rt4_scene_parse_frag(const char* text, size_t len, rt4_scene_desc* out, char* err, size_t errlen) {
  if (!out || (!text && len)) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  return parse_scene(std::string(text ? text : "", len), out, err, errlen);
}

extern "C" int rt4_scene_load_frag(const char* path, rt4_scene_desc* out, char* err, size_t errlen) {
  if (!path || !out) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return rt4_set_err(err, errlen, "cannot open scene file \"%s\"", path), RT4_ERR_IO;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  return parse_scene(s, out, err, errlen);
}
