/*
 * rt_scene.h — plain-data scene description shared by the host library
 * (librt_host.so), the HIP boundary (librt_hip.so) and the CPU oracle.
 *
 * Everything here is C, fp64, and owns nothing: pointers reference memory
 * owned by whoever filled the struct.  Field meanings follow the reference's
 * course types that the SoA flattening reads (mytracer.cpp:221-294):
 *   Vertex.position / Triangle.{i0,i1,i2,iuv0,iuv1,iuv2} / Mesh.{u,v}_coordinates_
 *   Mesh.material_ / Mesh.draw_mode_ / Mesh.texture_ / Light.{position,color}
 * Derived data (face normals, vertex normals, BVH) is NOT part of the raw
 * scene: the product host (C++) and the oracle (C) each derive it.
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Shading mode of a mesh; values as tested at mytracer_gpu.cu:498 and :501. */
enum { RT_DRAW_FLAT = 0, RT_DRAW_PHONG = 1 };

/* Phong material (course Material, fields read at mytracer.cpp:282-287). */
typedef struct rt_material {
  double ambient[3];
  double diffuse[3];
  double specular[3];
  double shininess;
  double mirror;      /* reflectivity in [0,1]; recursion only if > 0 (mytracer.cpp:547) */
  int shadowable;     /* receives shadows (mytracer.cpp:589); default 1 */
  int pad_;
} rt_material;

/* 8-bit RGB texture, row 0 = first row of the file (top), texel (x,y) at
 * rgb[3*(y*width+x)].  A texel value c is used as c/255.0 (fp64). */
typedef struct rt_texture {
  int width;                   /* <= 0: no texture (meshTexWidth_ == -1, mytracer.cpp:273) */
  int height;
  const unsigned char* rgb;
} rt_texture;

typedef struct rt_mesh {
  int n_vertices;
  const double* positions;     /* [3*n_vertices] */
  int n_triangles;
  const int* tri_vertex;       /* [3*n_triangles] mesh-local vertex ids (i0,i1,i2) */
  int n_uv;
  const double* u;             /* [n_uv] */
  const double* v;             /* [n_uv] */
  const int* tri_uv;           /* [3*n_triangles] mesh-local uv ids, or NULL when n_uv == 0 */
  int draw_mode;               /* RT_DRAW_FLAT / RT_DRAW_PHONG */
  int pad_;
  rt_material material;
  rt_texture texture;
} rt_mesh;

typedef struct rt_sphere {
  double center[3];
  double radius;
  rt_material material;
} rt_sphere;

typedef struct rt_plane {
  double center[3];
  double normal[3];            /* unit normal */
  rt_material material;
} rt_plane;

typedef struct rt_light {
  double position[3];
  double color[3];
} rt_light;

/* Camera as specified in a scene file: eye, look-at centre, up, vertical
 * field of view in degrees, image size (the course Camera constructor). */
typedef struct rt_camera_def {
  double eye[3];
  double center[3];
  double up[3];
  double fovy;
  int width;
  int height;
} rt_camera_def;

/* Derived pinhole camera: primary_ray(x,y) = Ray(eye, lower_left + x*x_dir +
 * y*y_dir - eye) (the [ABSENT] Camera::primary_ray called at
 * mytracer_gpu.cu:141/:208; semantics fixed in DESIGN.md §2). */
typedef struct rt_camera {
  double eye[3];
  double lower_left[3];
  double x_dir[3];
  double y_dir[3];
  int width;
  int height;
} rt_camera;

typedef struct rt_raw_scene {
  rt_camera_def camera;
  double background[3];
  double ambience[3];
  int max_depth;               /* number of reflection bounces after the primary hit */
  int n_lights;
  const rt_light* lights;
  int n_meshes;
  const rt_mesh* meshes;
  int n_spheres;
  const rt_sphere* spheres;
  int n_planes;
  const rt_plane* planes;
} rt_raw_scene;

#ifdef __cplusplus
}
#endif
#endif /* RT_SCENE_H */
