// BASELINE.json config 5: every primitive kind of shader.frag in one scene, tested in the order of
// shader.frag's find_intersection (:437-448): spaces, spheres, cylinders, cylinders union,
// hypercube, tiger. Progressive-accumulation workload (4K, many frames).

const vec3 sky_light = vec3(0.3, 0.5, 1.1);
const sun_properties sun = sun_properties(vec4(0.3, 1, 1, 0.2), PI * 0.07, vec3(800, 700, 300), 0.6);

const uint spaces_count = 2;
const visible_space[spaces_count] spaces = visible_space[spaces_count](
  visible_space(space(vec4(0, 0, -1.5, 0), vec4(0, 0, 1, 0)), material(0, 0.1, vec3(0.55, 0.5, 0.45))),
  visible_space(space(vec4(0, 9, 0, 0), vec4(0, 1, 0, 0)), material(0, 0.9, vec3(0.8, 0.85, 0.9)))
);

const uint spheres_count = 3;
const visible_sphere[spheres_count] spheres = visible_sphere[spheres_count](
  visible_sphere(sphere(vec4(-3.2, 4, -0.7, 0), 0.8), material(0, 0.85, vec3(0.9, 0.9, 0.9))),
  visible_sphere(sphere(vec4( 3.4, 5, 0.5, 0.3), 0.6), material(40, 0, vec3(1, 0.8, 0.5))),
  visible_sphere(sphere(vec4(0, 7, 2.2, -0.4), 0.9), material(0, 0.3, vec3(0.3, 0.4, 0.9)))
);

const uint cylinders_count = 1;
const visible_cylinder[cylinders_count] cylinders = visible_cylinder[cylinders_count](
  visible_cylinder(vec4(-2.5, 7, 0, 0), vec4(0, 0, 1, 0), vec4(0, 0, 0, 1), 0.35, material(0, 0.5, vec3(0.8, 0.6, 0.2)))
);

visible_cylinders_union cylinders_union = visible_cylinders_union(
  visible_cylinder(vec4(2.6, 3, -0.8, 0), vec4(1, 0, 0, 0), vec4(0, 0, 0, 1), 0.6, material(0, 0, vec3(1.0, 0.1, 0.1))),
  visible_cylinder(vec4(2.6, 3, -0.8, 0), vec4(0, 0, 1, 0), vec4(0, 1, 0, 0), 0.6, material(0, 0, vec3(0.1, 0.7, 0.3)))
);

visible_hypercube hypercube = init_hypercube(
  vec4(-1.4, 3.2, -0.9, 0),
  vec4(1, 0, 0, 0), vec4(0, 1, 0, 0), vec4(0, 0, 1, 0), vec4(0, 0, 0, 1),
  0.6,
  material(0, 0, vec3(0.72, 0.07, 0.20)), material(0, 0, vec3(0.00, 0.61, 0.28)),
  material(0, 0, vec3(1.00, 0.84, 0.00)), material(0, 0, vec3(0.40, 0.00, 0.80)),
  material(0, 0, vec3(1.00, 0.35, 0.00)), material(0, 0, vec3(0.00, 0.27, 0.68)),
  material(0, 0, vec3(1.00, 1.00, 1.00)), material(0, 0, vec3(0.01, 0.01, 0.01))
);

visible_tiger tiger = init_tiger(
  vec4(0.4, 5.5, 0.2, 0),
  vec4(1, 0, 0, 0), vec4(0, 0, 0, 1), vec4(0, 0, 1, 0), vec4(0, 1, 0, 0),
  0.7, 1.1,
  material(0, 0.2, vec3(0.9, 0.2, 0.1)), material(0, 0, vec3(0.1, 0.6, 0.9))
);

intersection find_intersection(ray ray) {
  intersection inter = NOT_INTERSECT;

  for (int i = 0; i < spaces.length(); i++)
    inter = closest(space_intersection(spaces[i], ray), inter);

  for (int i = 0; i < spheres.length(); i++)
    inter = closest(sphere_intersection(spheres[i], ray, true), inter);

  for (int i = 0; i < cylinders.length(); i++)
    inter = closest(cylinder_intersection(cylinders[i], ray, true), inter);

  inter = closest(cylinders_union_intersection(cylinders_union, ray), inter);
  inter = closest(hypercube_intersection(hypercube, ray), inter);
  inter = closest(tiger_intersection(tiger, ray), inter);

  return inter;
}
