// pbrt_scene.h — the .pbrt scene-file subset that feeds the photon-beam integrator on the GPU.
//
// Reference surface mirrored (bwiberg/beam-radiance-estimate-pbrt, pbrt-v3 fork):
//   tokenizer / grammar              src/core/pbrtlex.ll, src/core/pbrtparse.y (numbers via atof,
//                                    then (Float); "integer" values converted from the double)
//   ParamSet FindOne* / ReportUnused src/core/paramset.{h,cpp}
//   graphics state, CTM, media       src/core/api.cpp:765-1005 (Identity .. AttributeEnd),
//                                    :955-982 (MakeNamedMedium, MediumInterface), :1086-1157
//                                    (Material, MakeNamedMaterial, AreaLightSource, Shape)
//   Transform / Inverse / LookAt     src/core/transform.{h,cpp} (m and mInv tracked together)
//   MakeMedium                       src/core/api.cpp:547-593 (defaults, "scale", grid data2Medium)
//   camera medium                    api.cpp:651-655 (CreateMediumInterface at WorldEnd, outside)
//   film / camera / integrator       api.cpp:898-953 (parameters kept for the render)
//
// What the subset accepts is what the GPU scene model (include/bre_scene.h) can render; anything
// else is reported with pbrt-style Error()/Warning() text and the offending statement skipped:
//   * Shape "trianglemesh" -> one bre_triangle per index triple (vertices through the CTM exactly
//     as TriangleMesh does, mesh->p[i] = ObjectToWorld(P[i]), shapes/triangle.cpp; flip =
//     ReverseOrientation ^ TransformSwapsHandedness); any number up to BRE_MAX_SCENE_TRIANGLES (more
//     than BRE_MAX_TRIANGLES go through bre_scene.triangles_ext).
//   * Material "matte" with "Kd" (rgb, default 0.5) and sigma 0; MakeNamedMaterial/NamedMaterial.
//   * AreaLightSource "diffuse" ("L" x "scale", one-sided): every triangle of an emitting mesh is
//     its own light, as pbrtShape makes one DiffuseAreaLight per shape (api.cpp).
//   * media: "homogeneous" or "heterogeneous" (GridDensityMedium); the scene model has ONE medium
//     filling all space, so every shape's inside/outside medium and the camera medium must be
//     that medium (or all empty = vacuum).
//   * Camera "perspective" ("fov", lensradius 0) whose CTM is Identity followed by one LookAt.
//   * Film "image" (xresolution, yresolution, filename, scale); Integrator "photonbeam".
//   * Sampler / PixelFilter / Accelerator are accepted and ignored: the photon-beam integrator
//     draws from its own AwesomeSampler over HaltonSampler (photonbeam.cpp:456-462) and sets the
//     film image directly (Film::SetImage), so neither the scene's sampler nor filter is used.
//   * Include "file" (relative to the including file), comments, AttributeBegin/End,
//     TransformBegin/End, Translate, Scale, Rotate, LookAt, Transform, ConcatTransform,
//     CoordinateSystem, CoordSysTransform, ReverseOrientation.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/bre_scene.h"

namespace bre_host {

// One "type name" [values] parameter (pbrtparse.y ParamListItem after InitParamSet).
struct ParamItem {
    std::string type;  // integer float point3 vector3 normal rgb xyz spectrum bool string texture point2 ...
    std::string name;
    std::vector<float> floats;  // numeric values, converted from the double atof gave (Float)
    std::vector<int> ints;      // "integer" values
    std::vector<std::string> strings;
    std::vector<bool> bools;
    mutable bool lookedUp = false;
};

// pbrt::ParamSet subset (paramset.h): typed lookups with defaults, plus ReportUnused.
class ParamSet {
  public:
    void Add(ParamItem it);
    int FindOneInt(const std::string &name, int d) const;
    float FindOneFloat(const std::string &name, float d) const;
    bool FindOneBool(const std::string &name, bool d) const;
    std::string FindOneString(const std::string &name, const std::string &d) const;
    bool FindOnePoint3f(const std::string &name, float out[3]) const;
    // rgb / color only (RGBSpectrum::FromRGB copies); xyz is converted with XYZToRGB
    bool FindOneSpectrum(const std::string &name, float out[3]) const;
    const std::vector<float> *FindFloats(const std::string &name) const;
    const std::vector<int> *FindInts(const std::string &name) const;
    const std::vector<float> *FindPoint3fs(const std::string &name) const;
    bool Has(const std::string &name) const { return Find(name) != nullptr; }
    // names never looked up, "type name" each (paramset.cpp ReportUnused warns on them)
    std::vector<std::string> Unused() const;
    const std::vector<ParamItem> &Items() const { return items_; }

  private:
    const ParamItem *Find(const std::string &name) const;
    const ParamItem *FindTyped(const std::string &name, std::initializer_list<const char *> types) const;
    std::vector<ParamItem> items_;
};

// 4x4 matrix + tracked inverse, float arithmetic as pbrt's Transform (transform.{h,cpp}).
struct Xform {
    float m[4][4];
    float mInv[4][4];
    static Xform Identity();
    static Xform FromMatrix(const float rowMajor[4][4]);  // Transform(Matrix4x4): mInv = Inverse(m)
    static Xform Translate(float x, float y, float z);
    static Xform Scale(float x, float y, float z);
    static Xform Rotate(float thetaDeg, float ax, float ay, float az);
    static Xform LookAt(const float pos[3], const float look[3], const float up[3], bool *ok);
    Xform operator*(const Xform &t) const;
    Xform Inverse() const;  // pbrt Inverse(Transform): swaps m and mInv
    void ApplyPoint(const float p[3], float out[3]) const;
    bool IsIdentity() const;
};
// pbrt Matrix4x4 Inverse (Gauss-Jordan, full pivoting, transform.cpp:82-136); false if singular.
bool MatrixInverse(const float m[4][4], float out[4][4]);

struct FilmDesc {
    int xres = 1280, yres = 720;         // Film "image" defaults (film.cpp CreateFilm)
    std::string filename = "pbrt.pfm";   // "pbrt.exr" in the reference; this build writes PFM only
    float scale = 1.f;
};

// Everything the render needs from one .pbrt file.
struct PbrtScene {
    bre_scene scene;                  // grid_density / triangles_ext point into the vectors below
    std::vector<float> density;       // heterogeneous medium data (nx*ny*nz)
    std::vector<bre_triangle> triangles;  // the triangles when there are more than BRE_MAX_TRIANGLES
    // Re-point scene.grid_density / scene.triangles_ext at this object's vectors (after a copy).
    void Bind();
    FilmDesc film;
    std::string integratorName;       // "photonbeam" expected
    ParamSet integratorParams;        // CreatePhotonBeamIntegrator's ParamSet
    std::string cameraName;
    bool haveCamera = false;
    int errors = 0, warnings = 0;
    std::string messages;             // Error()/Warning() text, one message per line
};

// Parse a .pbrt file / string (pbrtParseFile / pbrtParseString).  Returns false only on a fatal
// problem (unreadable file, syntax error, no renderable scene); per-statement problems are
// recorded as errors and the statement skipped, as pbrt does.
bool ParsePbrtFile(const std::string &path, PbrtScene *out);
bool ParsePbrtString(const std::string &text, PbrtScene *out);

// Film::SetImage(L) + Film::WriteImage (film.cpp:132-140, 168-210) for the photon-beam
// integrator's image: per pixel RGB -> XYZ (RGBSpectrum::ToXYZ), filterWeightSum = 1, no splats,
// XYZ -> RGB, max(0, .) after the 1/weight multiply, + splatScale * 0, * scale.
void FilmFinalize(const float *L_rgb, int64_t npix, float scale, float *out_rgb);
// WriteImagePFM / ReadImagePFM (imageio.cpp:437-482): "PF", width height, -1 (little endian),
// rows bottom to top.  rgb is row-major from the top row.
bool WritePFM(const std::string &filename, const float *rgb, int width, int height, std::string *err);
bool ReadPFM(const std::string &filename, std::vector<float> *rgb, int *width, int *height, std::string *err);

}  // namespace bre_host
