/*
 * rt4.h — C ABI of the MI355X-native 4D path tracer (the drop-in boundary).
 *
 * The reference (BusyginIvan/4D_ray_tracing) has exactly one hot path: the per-cell trace loop of
 * executable/shader.frag (GLSL 330), driven by SFML through uniforms and one draw call per window.
 * This header replaces that boundary with plain C: POD structs, pointers and sizes, int status codes.
 *
 * Reference interface each entry point replaces (paths relative to the reference root):
 *   rt4_uniforms                  <- the 13 GLSL uniforms, executable/shader.frag:5-19, set through
 *                                    sf::Shader::setUniform in src/main.cpp:28-38,86-91 and
 *                                    src/windows/windows.cpp:41-44
 *   rt4_scene_desc                <- the scene block pasted into shader.frag (shader.frag:412-451,
 *                                    scenes/<name>.frag) + optional final_light override (shader.frag:454-468)
 *   rt4_scene_load_frag/parse     <- "paste a scene over shader.frag" workflow (executable/README.md:9-11),
 *                                    compiled at run time by sf::Shader::loadFromFile (src/main.cpp:26)
 *   rt4_properties_*              <- Properties (inc/properties.h:8-18, src/properties.cpp:12-77)
 *   rt4_orientation_update        <- Orientation::update (src/controls.cpp:72-86)
 *   rt4_uniforms_from_properties  <- initShader + first-frame uniforms (src/main.cpp:25-39,86-91),
 *                                    initControls (src/controls.cpp:140-159), CellsWindow
 *                                    (src/windows/windows.cpp:6-13,24-34)
 *   rt4_section_basis             <- ThreeWindowGroup::drawShaderImage (three_window_group.cpp:42-46)
 *   rt4_render_device / _host     <- CellsWindow::drawShaderImage -> texture.draw(sprite,&shader)
 *                                    (src/windows/windows.cpp:40-47): the "kernel launch"
 *
 * Conventions
 *   - Status: 0 = RT4_OK, negative = error; `err` (may be NULL) receives a NUL-terminated message.
 *     Nothing in the library aborts (the reference's error() aborts: src/util/util.cpp:9-12).
 *   - Images are float RGBA (16 B per pixel). Row 0 is the TOP of the displayed image, which in the
 *     reference is gl_FragCoord.y = 0.5 (RenderTexture::display() is never called).
 *   - The framebuffer is read (old_frame) and written in place by the lane that owns the pixel.
 *   - Re-entrant per (context, stream). One context per device per host thread.
 */
#ifndef RT4_H
#define RT4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT4_ABI_VERSION 2

enum rt4_status {
  RT4_OK = 0,
  RT4_ERR_ARG = -1,      /* bad argument / out-of-range value */
  RT4_ERR_IO = -2,       /* file cannot be opened or read */
  RT4_ERR_PARSE = -3,    /* properties or scene text not understood */
  RT4_ERR_HIP = -4,      /* HIP runtime error (no device, launch failure, ...) */
  RT4_ERR_CAPACITY = -5, /* scene exceeds the RT4_MAX_* limits below */
  RT4_ERR_PROPERTY = -6  /* missing key / bad value (reference: Properties::get* error paths) */
};

/* ---- uniforms: executable/shader.frag:5-19 (field-for-field) ------------------------------- */
typedef struct rt4_uniforms {
  int32_t seed;               /* shader.frag:5   (main.cpp:86, time based there; fixed here)    */
  int32_t samples;            /* shader.frag:6   ray_tracing.samples                          */
  int32_t reflections_amount; /* shader.frag:7   ray_tracing.reflections_amount               */
  float small_indent;         /* shader.frag:8   ray_tracing.small_indent                     */
  float resolution[2];        /* shader.frag:10  cells (windows.cpp:41)                       */
  float part;                 /* shader.frag:12  1/frameNumber (main.cpp:87)                  */
  float light_to_color_conversion_coefficient; /* shader.frag:13                            */
  float mtr_sizes[2];         /* shader.frag:16  (matrix_height*GOLDEN, matrix_height)        */
  float focus[4];             /* shader.frag:17                                               */
  float vec_to_mtr[4];        /* shader.frag:18  forward * focus_to_matrix_distance           */
  float top_drct[4];          /* shader.frag:19                                               */
  float right_drct[4];        /* shader.frag:19                                               */
} rt4_uniforms;

/* ---- scene: the primitive types of shader.frag:163-400 --------------------------------------- */
typedef struct rt4_material { /* shader.frag:163-167 */
  float glow;
  float refl_prob;
  float color[3];
} rt4_material;

typedef struct rt4_space { /* visible_space, shader.frag:225-228 */
  float point[4];
  float norm[4];
  rt4_material material;
} rt4_space;

typedef struct rt4_sphere { /* visible_sphere, shader.frag:189-192 */
  float center[4];
  float r;
  rt4_material material;
} rt4_sphere;

typedef struct rt4_cylinder { /* visible_cylinder, shader.frag:243-247 */
  float point[4];
  float axis1[4];
  float axis2[4];
  float r;
  rt4_material material;
} rt4_cylinder;

typedef struct rt4_cylinders_union { /* visible_cylinders_union, shader.frag:279-281 */
  rt4_cylinder cylinder1, cylinder2;
} rt4_cylinders_union;

typedef struct rt4_tiger { /* visible_tiger, shader.frag:298-300 (built by init_tiger :303-314) */
  rt4_cylinder inner_cyl1, outer_cyl1, inner_cyl2, outer_cyl2;
} rt4_tiger;

typedef struct rt4_cube { /* visible_cube, shader.frag:345-350 */
  float point[4]; /* space.point */
  float norm[4];  /* space.norm  */
  float x[4], y[4], z[4];
  float r;
  rt4_material material;
} rt4_cube;

typedef struct rt4_hypercube { /* visible_hypercube, shader.frag:370-372 (init_hypercube :374-392) */
  rt4_cube cubes[8];
} rt4_hypercube;

typedef struct rt4_sun { /* sun_properties, shader.frag:404-409 */
  float drct[4];
  float angular_size;
  float light[3];
  float sharpness;
} rt4_sun;

/* One statement `inter = closest(<group>_intersection(...), inter);` of find_intersection
 * (shader.frag:434-451). Groups are tested in array order; ties keep the accumulated hit. */
enum rt4_group_kind {
  RT4_GROUP_SPACES = 1,           /* for (i) space_intersection(spaces[i], ray)            :437-438 */
  RT4_GROUP_SPHERES = 2,          /* for (i) sphere_intersection(spheres[i], ray, outer)   :440-441 */
  RT4_GROUP_CYLINDERS = 3,        /* for (i) cylinder_intersection(cylinders[i], ray, outer) :443-444 */
  RT4_GROUP_CYLINDERS_UNION = 4,  /* cylinders_union_intersection(u, ray)                   :446 */
  RT4_GROUP_HYPERCUBE = 5,        /* hypercube_intersection(h, ray)                         :447 */
  RT4_GROUP_TIGER = 6             /* tiger_intersection(t, ray)                             :448 */
};

typedef struct rt4_group {
  int32_t kind;      /* rt4_group_kind */
  int32_t first;     /* index of the first object in the kind's array */
  int32_t count;     /* objects tested by this statement (1 for union/hypercube/tiger) */
  int32_t outer;     /* `outer` argument of sphere/cylinder tests (shader.frag:197,251) */
  int32_t new_first; /* 1: closest(new, inter) (reference form: tie keeps inter);
                        0: closest(inter, new) (tie takes the new hit) */
} rt4_group;

#define RT4_MAX_GROUPS 16
#define RT4_MAX_SPACES 32
#define RT4_MAX_SPHERES 32
#define RT4_MAX_CYLINDERS 16
#define RT4_MAX_UNIONS 4
#define RT4_MAX_HYPERCUBES 4
#define RT4_MAX_TIGERS 4

enum rt4_final_light_mode {
  RT4_FINAL_LIGHT_SUN_SKY = 0, /* default final_light, shader.frag:454-468 */
  RT4_FINAL_LIGHT_CONSTANT = 1 /* override returning a constant vec3 (S-room: scenes/Комната...:38-40) */
};

typedef struct rt4_scene_desc {
  float sky_light[3];         /* shader.frag:414 */
  rt4_sun sun;                /* shader.frag:415 */
  int32_t final_light_mode;   /* rt4_final_light_mode */
  float final_light_const[3]; /* value returned by a constant override */
  int32_t n_groups;
  rt4_group groups[RT4_MAX_GROUPS];
  int32_t n_spaces;
  rt4_space spaces[RT4_MAX_SPACES];
  int32_t n_spheres;
  rt4_sphere spheres[RT4_MAX_SPHERES];
  int32_t n_cylinders;
  rt4_cylinder cylinders[RT4_MAX_CYLINDERS];
  int32_t n_unions;
  rt4_cylinders_union unions[RT4_MAX_UNIONS];
  int32_t n_hypercubes;
  rt4_hypercube hypercubes[RT4_MAX_HYPERCUBES];
  int32_t n_tigers;
  rt4_tiger tigers[RT4_MAX_TIGERS];
} rt4_scene_desc;

/* ---- library info ------------------------------------------------------------------------- */
int rt4_abi_version(void);
const char* rt4_build_info(void); /* "rt4 <ver> gfx950 hip <ver> ..." */
size_t rt4_scene_desc_size(void); /* sizeof(rt4_scene_desc), for binding-layout checks */
size_t rt4_uniforms_size(void);

/* ---- properties.txt (src/properties.cpp:12-77) --------------------------------------------- */
typedef struct rt4_properties rt4_properties;
int rt4_properties_load(const char* path, rt4_properties** out, char* err, size_t errlen);
int rt4_properties_parse(const char* text, size_t len, rt4_properties** out, char* err, size_t errlen);
void rt4_properties_free(rt4_properties* p);
int rt4_properties_has(const rt4_properties* p, const char* key);
/* getString: copies the value (truncated to buflen-1); *needed receives strlen(value) if non-NULL */
int rt4_properties_get_string(const rt4_properties* p, const char* key, char* buf, size_t buflen,
                              size_t* needed, char* err, size_t errlen);
int rt4_properties_get_int(const rt4_properties* p, const char* key, int32_t* out, char* err, size_t errlen);
int rt4_properties_get_uint(const rt4_properties* p, const char* key, uint32_t* out, char* err, size_t errlen);
int rt4_properties_get_float(const rt4_properties* p, const char* key, float* out, char* err, size_t errlen);
int rt4_properties_get_bool(const rt4_properties* p, const char* key, int* out, char* err, size_t errlen);

/* ---- camera (src/controls.cpp:64-86) ------------------------------------------------------- */
typedef struct rt4_orientation {
  float forward[4], top[4], right[4], w_drct[4];
  float horizontal_forward[4], horizontal_right[4], vertical_top[4];
} rt4_orientation;
/* angles in radians (the reference converts degrees with convertDegreesToRadians, math.cpp:29) */
void rt4_orientation_update(float fi, float te, float psi, rt4_orientation* out);

enum rt4_section { /* three_window_group.cpp:42-46 */
  RT4_SECTION_YXZ = 0, /* main window:  top_drct = top,    right_drct = right */
  RT4_SECTION_YWZ = 1, /* extra window: top_drct = top,    right_drct = w     */
  RT4_SECTION_YXW = 2  /* extra window: top_drct = w,      right_drct = right */
};
int rt4_section_basis(const rt4_orientation* o, int section, float top[4], float right[4]);

/* Builds every uniform the reference host sets for the first frame of a still camera:
 * samples/reflections/indent/k/mtr_sizes (main.cpp:28-38), focus + vec_to_mtr (main.cpp:88-91,
 * controls.cpp:151-158), top/right for `section` and resolution = cells (windows.cpp:41-44),
 * part = 1 (frameNumber 1), seed = 0. cells_w/cells_h are the render resolution. */
int rt4_uniforms_from_properties(const rt4_properties* p, int32_t cells_w, int32_t cells_h, int section,
                                 rt4_uniforms* out, rt4_orientation* orientation_out, char* err,
                                 size_t errlen);
/* cells of a window: width/cell_size, (width/GOLDEN)/cell_size (windows.cpp:6-13,25-26);
 * window_type is "main" or "additional" (keys window.<type>.width / .cell_size). */
int rt4_window_cells(const rt4_properties* p, const char* window_type, int32_t* cells_w, int32_t* cells_h,
                     char* err, size_t errlen);

/* ---- camera model: SphOrientation, mouse / wheel / WASD-EQ motion (src/controls.cpp) ---------- */
typedef struct rt4_camera {
  float fi, te, psi;                       /* radians, normalised (SphOrientation, controls.cpp:25-54) */
  float psi_range_center, psi_range_radius;
  int32_t constrain_psi_range;
  float mouse_sensitivity, wheel_sensitivity, movement_speed; /* controls.cpp:144-147 */
  float focus_to_matrix_distance;          /* main.cpp:73 */
  float focus[4];                          /* controls.cpp:150-156 */
  uint32_t frame_number;                   /* frames since the camera last changed, from 1 (main.cpp:72) */
  rt4_orientation orientation;             /* Orientation::update() of (fi, te, psi) */
} rt4_camera;

/* Movement keys held during a frame (controls.cpp:98-113). */
enum rt4_move_key {
  RT4_KEY_FORWARD = 1,  /* W      horizontal_forward */
  RT4_KEY_BACK = 2,     /* S     -horizontal_forward */
  RT4_KEY_RIGHT = 4,    /* D      horizontal_right   */
  RT4_KEY_LEFT = 8,     /* A     -horizontal_right   */
  RT4_KEY_UP = 16,      /* Space  vertical_top       */
  RT4_KEY_DOWN = 32,    /* LShift -vertical_top      */
  RT4_KEY_W_POS = 64,   /* E      w_drct             */
  RT4_KEY_W_NEG = 128   /* Q     -w_drct             */
};

/* initControls + SphOrientation::init (controls.cpp:140-159, :29-39): angles from degrees, psi range,
 * sensitivities, speed, focus; frame_number = 1. */
int rt4_camera_init(const rt4_properties* p, rt4_camera* cam, char* err, size_t errlen);
/* changeFi / changeTe / changePsi (each re-normalises) + Orientation::update + frame_number = 1
 * (controls.cpp:51-53, :186-198). */
void rt4_camera_rotate(rt4_camera* cam, float d_fi, float d_te, float d_psi);
/* Event::MouseMoved with the cursor (dx, dy) from the window centre, dy up (controls.cpp:181-193):
 * returns 1 and changes nothing when |dx| or |dy| exceeds max_offset (the cursor is re-centred),
 * 0 after rotating by (dx, dy) * mouse_sensitivity (a zero move changes nothing). */
int rt4_camera_mouse_move(rt4_camera* cam, int32_t dx, int32_t dy, uint32_t max_offset);
/* Event::MouseWheelScrolled: psi += delta * wheel_sensitivity (controls.cpp:196-201). */
void rt4_camera_wheel(rt4_camera* cam, float delta);
/* move(seconds) (controls.cpp:118-134): focus += drct * (seconds * movement_speed / |drct|) for the
 * sum drct of the held keys' directions; frame_number = 1 when it moved. */
void rt4_camera_move(rt4_camera* cam, uint32_t keys, float seconds);
/* Uniforms of the next frame (main.cpp:86-91, windows.cpp:41-44): base supplies samples,
 * reflections_amount, small_indent, k, mtr_sizes and resolution; then seed, part = 1/frame_number,
 * focus, vec_to_mtr = forward * focus_to_matrix_distance and top/right of `section`. Advances
 * frame_number (frameNumber++). */
int rt4_camera_frame_uniforms(rt4_camera* cam, const rt4_uniforms* base, int section, int32_t seed,
                              rt4_uniforms* out);

/* ---- image output (presentation; windows.cpp:24-53 shows frames in SFML windows instead) ------ */
/* Binary PPM (P6) of an RGBA frame in any rt4_frame_format, rows top first, alpha dropped; float
 * channels are clamped to [0, 1] and mapped with the RGBA8 rule u = (uint8)(v * 255 + 0.5). */
int rt4_write_ppm(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                  char* err, size_t errlen);
/* The same pixels as an 8-bit RGB PNG (uncompressed deflate blocks, so no zlib dependency); w <= 21844. */
int rt4_write_png(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                  char* err, size_t errlen);

/* ---- accumulator checkpoint / resume (no reference counterpart) ----------------
 * The reference keeps the progressive average only in the window's texture: old_frame is blended with
 * part = 1/frameNumber (main.cpp:86-91) and restarts at frameNumber = 1 when the camera moves
 * (controls.cpp:132,181,190). A checkpoint is that texture in its rt4_frame_format plus the number of
 * frames already blended and the base seed, so a resumed run (frames frames_done + 1, ... through
 * rt4_progressive_uniforms) continues the same blend bit for bit.
 * File (little-endian): "RT4ACC1\0", int32 version (2), w, h, format, int64 frames_done, uint32 seed,
 * uint32 key (rt4_accum_key of the run, 0 = not recorded; version-1 files hold 0 there and still load),
 * then h rows of w pixels, rows top first, no padding. A save writes <path>.tmp, flushes it to the disk and
 * renames it over path, so a failed save leaves the previous checkpoint intact. */
#define RT4_ACCUM_VERSION 2
int rt4_accum_save(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                   int64_t frames_done, uint32_t seed, char* err, size_t errlen);
/* rt4_accum_save with the run's key, so that a resume can refuse a checkpoint of another run. */
int rt4_accum_save_key(const char* path, const void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                       int64_t frames_done, uint32_t seed, uint32_t key, char* err, size_t errlen);
/* The run's key (never 0): a hash of the scene and of the uniforms that decide the progressive image other
 * than seed and part (samples, bounces, indent, tone-map coefficient, resolution, matrix, camera pose). */
uint32_t rt4_accum_key(const rt4_scene_desc* scene, const rt4_uniforms* u);
/* The key a checkpoint was saved with (0: not recorded). */
int rt4_accum_key_of(const char* path, uint32_t* key, char* err, size_t errlen);
/* Header only: any output pointer may be null. RT4_ERR_PARSE for a file that is not a checkpoint. */
int rt4_accum_info(const char* path, int32_t* w, int32_t* h, int32_t* format, int64_t* frames_done, uint32_t* seed,
                   char* err, size_t errlen);
/* Reads the pixels into a host frame of the checkpoint's w, h and format (RT4_ERR_ARG if the caller's
 * differ); the header fields as rt4_accum_info. */
int rt4_accum_load(const char* path, void* frame, int32_t format, int32_t w, int32_t h, int64_t row_stride_px,
                   int64_t* frames_done, uint32_t* seed, char* err, size_t errlen);

/* ---- scenes ------------------------------------------------------------------------------- */
/* Accepts a scene snippet (scenes/<name>.frag) or a whole shader.frag; UTF-8 paths. */
int rt4_scene_load_frag(const char* path, rt4_scene_desc* out, char* err, size_t errlen);
int rt4_scene_parse_frag(const char* text, size_t len, rt4_scene_desc* out, char* err, size_t errlen);
int rt4_scene_validate(const rt4_scene_desc* s, char* err, size_t errlen);
/* The reference's five scenes, rebuilt from their values (scenes/<name>.frag, executable/shader.frag):
 * "sphere" (Шар, плоскость и светилник), "room" (Комната со сферой), "tiger" (Фигура tiger; also
 * the shipped shader.frag default), "cylinder4d" (Четырёхмерный цилиндр), "hypercube" (Гиперкуб). */
int rt4_scene_builtin(const char* name, rt4_scene_desc* out, char* err, size_t errlen);

/* ---- device context + trace kernel --------------------------------------------------------- */
typedef struct rt4_context rt4_context;

/* Memoise w_by_volume (shader.frag:141-150) over its whole input domain: rand() yields only
 * 2^23 values (shader.frag:111-118), so a 32 MiB table built on the device at context creation
 * by the same device function reproduces every Newton result bit for bit. */
#define RT4_FLAG_SAMPLER_LUT 0x1u
/* Always use the generic find_intersection (any group list) instead of the kernel specialised for
 * the scene's shape. Results are identical; used by the tests to cover both code paths. */
#define RT4_FLAG_GENERIC_KERNEL 0x2u
/* Primary-ray reuse. Every sample of a pixel starts with the same primary ray (shader.frag:519-521),
 * so find_intersection of that ray has the same result in all of them: the kernel evaluates it once
 * per pixel and starts every later sample from the cached candidate (shaded with the sample's own
 * random numbers, in the iteration that ended the previous sample). Images and the d_counter count
 * (find_intersection calls of the reference) are unchanged; rt4_context_evaluated reports the calls
 * actually evaluated. Specialised kernels only (ignored with RT4_FLAG_GENERIC_KERNEL or a generic
 * scene). SURVEY.md 8(d): a rate measured with it is labelled reference-equivalent. */
#define RT4_FLAG_PRIMARY_REUSE 0x4u
/* Overlapped launches (the default). A single-frame launch (rt4_render_device[_ex],
 * rt4_render_sections_device) runs its trace kernel on a context-owned side stream and writes the frame's light
 * sums to a context-owned slot buffer; only the blend into the frame (and the count) runs on the caller's stream.
 * Back-to-back frames (a moving camera, main.cpp:93; the 4D view's three sections, three_window_group.cpp:42-46)
 * then overlap each frame's trace with the previous frames' drain. Stream semantics are unchanged: the frame and
 * the counter are written in the caller's stream order; images and counts are identical to serial launches.
 * Depth and memory: a launch with fewer 8x8 tiles than the chip holds waves (~7000 tiles: the 4D view's sections
 * at properties.txt sizes) keeps up to 8 launches in flight on 8 side streams with 8 slot buffers; any larger one
 * up to 3, with 3 buffers. A slot buffer is 16 B per pixel of the largest launch it served: a 1080p frame uses
 * 3 x 33 MB, a 4K frame 3 x 133 MB, small frames at most 8 x 7.3 MB (rt4_context_overlap_bytes). The first launch
 * that needs a larger buffer waits on the host for the launches in flight and allocates it
 * (rt4_context_reserve_overlap does that ahead of time); if the allocation fails, that frame runs serially.
 * Hardware queues: the 8 side streams of the deep overlap share HIP's default four hardware queues per process;
 * set GPU_MAX_HW_QUEUES=8 in the environment before the process first touches HIP to give each its own (the 4D
 * view loop on config 2's scene: 0.25 ms per frame with the default, 0.17 ms with 8; frames that fill the chip
 * are unaffected). */
/* Every launch runs entirely on the caller's stream (no side streams, no slot buffers). */
#define RT4_FLAG_SERIAL_FRAMES 0x8u
/* Caps the overlap at 3 launches in flight for every frame size (3 side streams, 3 slot buffers): for processes
 * that keep HIP's four hardware queues or want the smaller footprint. Images and counts are unchanged. */
#define RT4_FLAG_OVERLAP_SHALLOW 0x10u

int rt4_context_create(int device, uint32_t flags, rt4_context** out, char* err, size_t errlen);
/* Uploads a scene (the reference recompiles the shader: src/main.cpp:25-39). Waits for the
 * context's launches still in flight on any stream before it replaces the device copy, so a frame
 * issued earlier renders the previous scene. Scene constants are verified on the device once per
 * process (cached by bit pattern), so setting a scene seen before costs only the upload. */
int rt4_context_set_scene(rt4_context* ctx, const rt4_scene_desc* scene, char* err, size_t errlen);
void rt4_context_destroy(rt4_context* ctx);

/* Pixel set of one launch (w <= 65535, h <= 16383). Local row i in [0,h) maps to image row
 *   band_rows == 0 : y0 + i
 *   band_rows  > 0 : y0 + (i / band_rows) * band_step + (i % band_rows)
 * and local column j in [0,w) to image column x0 + j. Scene coordinates come from the full image
 * size in uniforms.resolution, so any partition renders exactly the pixels of the whole image. */
typedef struct rt4_region {
  int32_t x0, y0, w, h;
  int32_t band_rows;
  int32_t band_step;
} rt4_region;

/* d_rgba: device float4 framebuffer; pixel (i, j) at d_rgba + 4*(i*row_stride_px + j).
 * Holds old_frame on entry and mix(old, new, part) on return (shader.frag:524-527).
 * d_counter (may be NULL): device uint64 incremented by the number of find_intersection calls
 * (one per ray-bounce, shader.frag:475). stream: hipStream_t (NULL = default stream).
 * Asynchronous: no host synchronisation and no allocation once the context's buffers hold the launch: the
 * tile-order buffer covers 2^18 8x8 tiles (16.7 M pixels; a larger launch grows it once) and the overlap's slot
 * buffers grow to the largest frame seen (without RT4_FLAG_SERIAL_FRAMES, the default: the first launch of a larger
 * frame waits for the launches in flight and allocates; rt4_context_reserve_overlap does it ahead of time; a
 * serial context has no slot buffers). Launches of one
 * context run in submission order: a launch on another stream than the previous one waits for it. */
int rt4_render_device(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* d_rgba,
                      int64_t row_stride_px, unsigned long long* d_counter, void* stream, char* err,
                      size_t errlen);

/* Host-buffer convenience wrapper: copies rgba (same layout) to the device, renders, copies back,
 * synchronises. n_intersections (may be NULL) receives the count. */
int rt4_render_host(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* rgba,
                    int64_t row_stride_px, uint64_t* n_intersections, char* err, size_t errlen);

/* ---- frame formats, progressive accumulation, batched sections --------- */
/* What old_frame / gl_FragColor live in. The blend mix(old, new, part) (shader.frag:524-527) is
 * always evaluated in fp32 (one fma per channel); only the stored value differs. */
enum rt4_frame_format {
  RT4_FRAME_RGBA32F = 0, /* float4, 16 B/pixel (rt4_render_device) */
  RT4_FRAME_RGBA16F = 1, /* IEEE half x4, 8 B/pixel: fp16 accumulator, stored round-to-nearest-even */
  RT4_FRAME_RGBA8 = 2    /* unorm8 x4, 4 B/pixel: the reference's RenderTexture (windows.cpp:31), which
                          * quantises old_frame every frame: old = u / 255.0f, stored
                          * u = (uint8_t)(min(max(v, 0), 1) * 255.0f + 0.5f), alpha 255 */
};
/* Bytes per pixel of a format; 0 if unknown. */
int32_t rt4_frame_format_bytes(int32_t format);

/* rt4_render_device for any frame format: d_frame holds h rows of row_stride_px pixels of the
 * format's size. */
int rt4_render_device_ex(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, void* d_frame,
                         int32_t format, int64_t row_stride_px, unsigned long long* d_counter, void* stream,
                         char* err, size_t errlen);
int rt4_render_host_ex(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, void* frame,
                       int32_t format, int64_t row_stride_px, uint64_t* n_intersections, char* err,
                       size_t errlen);

/* Progressive accumulation (main.cpp:72,86-88): frame_number counts frames since the camera last
 * moved, from 1. part = 1.0f / frame_number (frame 1 overwrites old_frame). The reference draws
 * a fresh time-based seed every frame (main.cpp:52-54,86); this deterministic replacement is
 * seed_n = base->seed ^ (frame_number * 0x9E3779B9). */
int rt4_progressive_uniforms(const rt4_uniforms* base, uint32_t frame_number, rt4_uniforms* out);

/* Up to three images in ONE launch: the sections of ThreeWindowGroup::drawShaderImage
 * (three_window_group.cpp:42-46; bases from rt4_section_basis). Per job: resolution, mtr_sizes,
 * vec_to_mtr, top_drct, right_drct, the region and the frame. seed, samples, reflections_amount,
 * small_indent, part, light_to_color_conversion_coefficient and focus must equal jobs[0]'s (one
 * shader, one frame; RT4_ERR_ARG otherwise). Each image equals its own rt4_render_device_ex bit for
 * bit; the pixel queue is shared, so the sections balance each other. Region h <= 16383 here. */
#define RT4_MAX_SECTIONS 3
typedef struct rt4_section_job {
  rt4_uniforms u;
  rt4_region region;
  void* d_frame;
  int64_t row_stride_px;
} rt4_section_job;
int rt4_render_sections_device(rt4_context* ctx, const rt4_section_job* jobs, int32_t n_jobs, int32_t format,
                               unsigned long long* d_counter, void* stream, char* err, size_t errlen);

/* n_frames consecutive frames into the same frame buffer, pipelined: the same result, bit for bit, as
 * n_frames calls of rt4_render_device_ex with u[0], u[1], ... in order (the frame loop of main.cpp:57-111
 * while the camera rests: progressive accumulation, or a benchmark loop), and d_counter receives the
 * sum of their counts. u[f] may differ from u[0] only in seed and part (rt4_progressive_uniforms);
 * RT4_ERR_ARG otherwise. The frames share one pixel queue (item = frame x 8x8 tile), so the drain at the
 * end of a launch (each lane finishing its last pixel's samples in order) is paid once per up to
 * RT4_MAX_FRAMES frames instead of once per frame. Each pixel's tone-mapped colour of every frame goes
 * to a context-owned scratch buffer (16 B per pixel and frame, up to 4 GiB: the frames are split into
 * launches that fit), then one pass blends the frames in order into d_frame with the same per-frame ops
 * and roundings as rt4_render_device_ex. The intermediate frames are not stored in d_frame. Regions
 * wider or taller than 8191 pixels run frame by frame. Asynchronous like rt4_render_device_ex; the first
 * call with a larger scratch need allocates (synchronises the stream once). */
#define RT4_MAX_FRAMES 64
int rt4_render_frames_device(rt4_context* ctx, const rt4_uniforms* u, int32_t n_frames, const rt4_region* region,
                             void* d_frame, int32_t format, int64_t row_stride_px, unsigned long long* d_counter,
                             void* stream, char* err, size_t errlen);
/* Allocates (and first-touches) the frame-colour scratch that pipelined launches of a w x h region use,
 * so that the first rt4_render_frames_device call of that size neither allocates nor synchronises.
 * Waits for the context's launches in flight when it has to grow the buffer. */
int rt4_context_reserve_frames(rt4_context* ctx, int32_t w, int32_t h, char* err, size_t errlen);
/* Frames per pipelined launch rt4_render_frames_device uses for a w x h region with the context's
 * current scene (1: frame by frame). The mirror-room tiger kernel (three or more spaces and a tiger)
 * runs frame by frame: it measured slower pipelined. */
int32_t rt4_context_frames_per_launch(const rt4_context* ctx, int32_t w, int32_t h);

/* ---- multi-GPU pixel bands (replaces the one whole-texture draw of windows.cpp:45) ---
 * A width x height frame is cut into bands of `band` rows (the last one may be short) dealt round-robin
 * over `world` ranks, so every rank gets the same mix of cheap sky rows and expensive object rows. Every
 * pixel is independent (shader.frag:104-108: the RNG depends only on the pixel, the seed and its own call
 * counter), so the assembled image equals a one-GPU render bit for bit.
 * rt4_band_plan: the region of `rank` (band layout of rt4_region; h = 0 when the rank owns no band) and
 * rows_max, the rows of the largest shard (>= 1): every rank renders into a buffer of rows_max rows of
 * width pixels, so one ncclGather of equal-size shards collects them (4d_ray_tracing_amd/shard.py
 * make_plan is the same arithmetic). RT4_ERR_ARG for width, height, world or band < 1, or rank outside
 * [0, world). */
int rt4_band_plan(int32_t width, int32_t height, int32_t world, int32_t band, int32_t rank, rt4_region* region,
                  int32_t* rows_max, char* err, size_t errlen);
/* Assembles the frame on the root from the gathered shards: d_gathered holds world x rows_max rows of
 * width pixels, rank-major (what ncclGather leaves on the root), d_image receives height rows of width
 * pixels (row stride width); pixel size rt4_frame_format_bytes(format). Asynchronous on stream (a
 * hipStream_t of the device that holds both buffers). */
int rt4_bands_unpermute_device(const void* d_gathered, void* d_image, int32_t width, int32_t height, int32_t world,
                               int32_t band, int32_t rows_max, int32_t format, void* stream, char* err, size_t errlen);

/* ---- diagnostics (used by the parity tests; not on the render path) ------------------------- */
/* Bytes of the context's frame-colour scratch for pipelined frames (0 before any pipelined launch or
 * reservation; a scene that runs frame by frame never allocates it). */
uint64_t rt4_context_frame_scratch_bytes(const rt4_context* ctx);
/* Bytes of the context's overlap slot buffers (without RT4_FLAG_SERIAL_FRAMES, the default: 0 before any single-frame
 * launch or reservation; a context made with RT4_FLAG_SERIAL_FRAMES always returns 0). */
uint64_t rt4_context_overlap_bytes(const rt4_context* ctx);
/* Allocates the slot buffers that overlapped single-frame launches of one w x h image use with the context's
 * current scene (3, or 8 for a frame too small to fill the chip), so that the first such launch neither
 * allocates nor synchronises. Waits for the context's launches in flight when it grows a buffer. A no-op for a
 * context made with RT4_FLAG_SERIAL_FRAMES. For the 4D view's sections pass w x h with w * h >= the sections'
 * pixels together. */
int rt4_context_reserve_overlap(rt4_context* ctx, int32_t w, int32_t h, char* err, size_t errlen);
enum rt4_eval_fn {
  RT4_EVAL_ACOS = 0, RT4_EVAL_ASIN = 1, RT4_EVAL_SIN = 2, RT4_EVAL_COS = 3,
  RT4_EVAL_VOLUME_BY_W = 4, /* shader.frag:136-138 */
  RT4_EVAL_W_BY_VOLUME = 5, /* shader.frag:141-150; aux[i] = Newton iterations */
  RT4_EVAL_HASH = 6,        /* shader.frag:94-102 on the bit pattern of in[i] */
  RT4_EVAL_SQRT = 7         /* the kernel's correctly rounded sqrt (GLSL sqrt, e.g. :47, :137, :216) */
};
/* Evaluates a device math function element-wise (synchronous; host buffers). */
int rt4_debug_eval(rt4_context* ctx, int fn, const float* in, float* out, int32_t* aux, int64_t n, char* err,
                   size_t errlen);

/* Runs find_intersection (shader.frag:434-451) for n rays of the context's scene on the device.
 * rays: n x 8 floats (point xyzw, drct xyzw). out: n x 8 floats {hit(0/1), dist, norm xyzw,
 * glow, refl_prob}; out_color: n x 3 floats. Synchronous; host buffers. */
int rt4_debug_find_intersection(rt4_context* ctx, const float* rays, float* out, float* out_color, int64_t n,
                                char* err, size_t errlen);

/* Counts the 32-bit patterns x for which the kernel's sqrt (fast path without input scaling) differs
 * from the IEEE square root; 0 expected. Exhaustive over all 2^32 inputs on the device (~10 ms). */
int rt4_debug_verify_sqrt(rt4_context* ctx, uint64_t* mismatches, char* err, size_t errlen);

/* find_intersection calls the context's launches actually evaluated since the last reset (all of them
 * unless RT4_FLAG_PRIMARY_REUSE: only its launches count). Waits for the context's last launch. */
int rt4_context_evaluated(rt4_context* ctx, uint64_t* n, int32_t reset, char* err, size_t errlen);

/* The scene-constant checks of rt4_context_set_scene, alone (synchronous). verify_div: mismatches of
 * the verified-divisor quotient against x / b over the reduced sweep (full = 0: positive numerators,
 * edge exponents + three of the middle band) or over all 2^32 numerators (full = 1);
 * set_scene enables the fast quotient iff the reduced count is 0. sky_threshold: the smallest float c
 * with acos(c) < ang in the kernel's acos (NaN: none), over c in (0.5, 1] for ang <= 1 (full = 0) or
 * over all 2^32 patterns (full = 1). */
int rt4_debug_verify_div(rt4_context* ctx, float b, int32_t full, uint64_t* mismatches, char* err, size_t errlen);
int rt4_debug_sky_threshold(rt4_context* ctx, float ang, int32_t full, float* c_min, char* err, size_t errlen);

/* Trace kernel selected for the context's scene: 0xFFFFFFFF = the generic find_intersection
 * (any group list); otherwise the K_* group bits (low byte: 1 spaces, 2 spheres, 4 cylinders,
 * 8 union, 16 hypercube, 32 tiger), plus (n_spaces+1) << 8 | (n_spheres+1) << 16 |
 * (n_cylinders+1) << 24 when a kernel compiled for the scene's exact object counts exists.
 * 0 if the context has no scene. */
uint32_t rt4_context_kernel_shape(const rt4_context* ctx);

#ifdef __cplusplus
}
#endif

#endif /* RT4_H */
