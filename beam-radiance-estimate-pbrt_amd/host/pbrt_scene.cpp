// pbrt_scene.cpp — see pbrt_scene.h.
#include "pbrt_scene.h"

#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <utility>

namespace bre_host {

// ---------------------------------------------------------------------------------------------
// ParamSet (paramset.cpp)

void ParamSet::Add(ParamItem it) {
    for (auto &e : items_)
        if (e.name == it.name) {  // paramset.cpp EraseX + AddX: a later value replaces an earlier one
            e = std::move(it);
            return;
        }
    items_.push_back(std::move(it));
}

const ParamItem *ParamSet::Find(const std::string &name) const {
    for (auto &e : items_)
        if (e.name == name) return &e;
    return nullptr;
}

const ParamItem *ParamSet::FindTyped(const std::string &name, std::initializer_list<const char *> types) const {
    for (auto &e : items_) {
        if (e.name != name) continue;
        for (const char *t : types)
            if (e.type == t) {
                e.lookedUp = true;
                return &e;
            }
    }
    return nullptr;
}

int ParamSet::FindOneInt(const std::string &name, int d) const {
    const ParamItem *p = FindTyped(name, {"integer"});
    return (p && p->ints.size() == 1) ? p->ints[0] : d;
}

float ParamSet::FindOneFloat(const std::string &name, float d) const {
    const ParamItem *p = FindTyped(name, {"float"});
    return (p && p->floats.size() == 1) ? p->floats[0] : d;
}

bool ParamSet::FindOneBool(const std::string &name, bool d) const {
    const ParamItem *p = FindTyped(name, {"bool"});
    return (p && p->bools.size() == 1) ? (bool)p->bools[0] : d;
}

std::string ParamSet::FindOneString(const std::string &name, const std::string &d) const {
    const ParamItem *p = FindTyped(name, {"string"});
    return (p && p->strings.size() == 1) ? p->strings[0] : d;
}

bool ParamSet::FindOnePoint3f(const std::string &name, float out[3]) const {
    const ParamItem *p = FindTyped(name, {"point3"});
    if (!p || p->floats.size() != 3) return false;
    for (int k = 0; k < 3; ++k) out[k] = p->floats[k];
    return true;
}

bool ParamSet::FindOneSpectrum(const std::string &name, float out[3]) const {
    const ParamItem *p = FindTyped(name, {"rgb", "xyz"});
    if (!p || p->floats.size() != 3) return false;
    if (p->type == "rgb") {
        for (int k = 0; k < 3; ++k) out[k] = p->floats[k];
    } else {  // XYZToRGB (spectrum.h:56-60)
        const float *x = p->floats.data();
        out[0] = 3.240479f * x[0] - 1.537150f * x[1] - 0.498535f * x[2];
        out[1] = -0.969256f * x[0] + 1.875991f * x[1] + 0.041556f * x[2];
        out[2] = 0.055648f * x[0] - 0.204043f * x[1] + 1.057311f * x[2];
    }
    return true;
}

const std::vector<float> *ParamSet::FindFloats(const std::string &name) const {
    const ParamItem *p = FindTyped(name, {"float"});
    return p ? &p->floats : nullptr;
}

const std::vector<int> *ParamSet::FindInts(const std::string &name) const {
    const ParamItem *p = FindTyped(name, {"integer"});
    return p ? &p->ints : nullptr;
}

const std::vector<float> *ParamSet::FindPoint3fs(const std::string &name) const {
    const ParamItem *p = FindTyped(name, {"point3"});
    return p ? &p->floats : nullptr;
}

std::vector<std::string> ParamSet::Unused() const {
    std::vector<std::string> u;
    for (auto &e : items_)
        if (!e.lookedUp) u.push_back("\"" + e.type + " " + e.name + "\"");
    return u;
}

// ---------------------------------------------------------------------------------------------
// Transforms (transform.{h,cpp}), float arithmetic in pbrt's operation order

static void MatMul(const float a[4][4], const float b[4][4], float r[4][4]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r[i][j] = a[i][0] * b[0][j] + a[i][1] * b[1][j] + a[i][2] * b[2][j] + a[i][3] * b[3][j];
}

static void MatIdentity(float m[4][4]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) m[i][j] = i == j ? 1.f : 0.f;
}

static void MatTranspose(const float m[4][4], float t[4][4]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) t[i][j] = m[j][i];
}

bool MatrixInverse(const float m[4][4], float out[4][4]) {
    int indxc[4], indxr[4];
    int ipiv[4] = {0, 0, 0, 0};
    float minv[4][4];
    memcpy(minv, m, sizeof(minv));
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        float big = 0.f;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] == 1) continue;
            for (int k = 0; k < 4; k++) {
                if (ipiv[k] == 0) {
                    if (std::abs(minv[j][k]) >= big) {
                        big = std::abs(minv[j][k]);
                        irow = j;
                        icol = k;
                    }
                } else if (ipiv[k] > 1) {
                    return false;
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(minv[irow][k], minv[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (minv[icol][icol] == 0.f) return false;
        const float pivinv = (float)(1. / minv[icol][icol]);  // double divide, stored as Float
        minv[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j == icol) continue;
            const float save = minv[j][icol];
            minv[j][icol] = 0;
            for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
        }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(minv[k][indxr[j]], minv[k][indxc[j]]);
    memcpy(out, minv, sizeof(minv));
    return true;
}

Xform Xform::Identity() {
    Xform t;
    MatIdentity(t.m);
    MatIdentity(t.mInv);
    return t;
}

Xform Xform::FromMatrix(const float rm[4][4]) {
    Xform t;
    memcpy(t.m, rm, sizeof(t.m));
    if (!MatrixInverse(t.m, t.mInv)) {
        // pbrt prints "Singular matrix in MatrixInvert" and carries on with the partial result;
        // a singular CTM is useless for this scene model, so keep a NaN inverse that fails checks
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) t.mInv[i][j] = NAN;
    }
    return t;
}

Xform Xform::Translate(float x, float y, float z) {
    Xform t = Identity();
    t.m[0][3] = x;
    t.m[1][3] = y;
    t.m[2][3] = z;
    t.mInv[0][3] = -x;
    t.mInv[1][3] = -y;
    t.mInv[2][3] = -z;
    return t;
}

Xform Xform::Scale(float x, float y, float z) {
    Xform t = Identity();
    t.m[0][0] = x;
    t.m[1][1] = y;
    t.m[2][2] = z;
    t.mInv[0][0] = 1 / x;
    t.mInv[1][1] = 1 / y;
    t.mInv[2][2] = 1 / z;
    return t;
}

static void Normalize3(const float v[3], float out[3]) {
    const float len = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const float inv = 1 / len;  // Vector3 operator/ multiplies by 1/f (geometry.h)
    for (int k = 0; k < 3; ++k) out[k] = v[k] * inv;
}

static void Cross3(const float a[3], const float b[3], float out[3]) {
    // geometry.h Cross: evaluated in double, rounded once per component
    const double ax = a[0], ay = a[1], az = a[2], bx = b[0], by = b[1], bz = b[2];
    out[0] = (float)((ay * bz) - (az * by));
    out[1] = (float)((az * bx) - (ax * bz));
    out[2] = (float)((ax * by) - (ay * bx));
}

Xform Xform::Rotate(float theta, float ax, float ay, float az) {
    const float axis[3] = {ax, ay, az};
    float a[3];
    Normalize3(axis, a);
    const float rad = (float)(3.14159265358979323846f / 180) * theta;  // Radians (pbrt.h:298)
    const float s = std::sin(rad), c = std::cos(rad);
    Xform t = Identity();
    t.m[0][0] = a[0] * a[0] + (1 - a[0] * a[0]) * c;
    t.m[0][1] = a[0] * a[1] * (1 - c) - a[2] * s;
    t.m[0][2] = a[0] * a[2] * (1 - c) + a[1] * s;
    t.m[0][3] = 0;
    t.m[1][0] = a[0] * a[1] * (1 - c) + a[2] * s;
    t.m[1][1] = a[1] * a[1] + (1 - a[1] * a[1]) * c;
    t.m[1][2] = a[1] * a[2] * (1 - c) - a[0] * s;
    t.m[1][3] = 0;
    t.m[2][0] = a[0] * a[2] * (1 - c) - a[1] * s;
    t.m[2][1] = a[1] * a[2] * (1 - c) + a[0] * s;
    t.m[2][2] = a[2] * a[2] + (1 - a[2] * a[2]) * c;
    t.m[2][3] = 0;
    MatTranspose(t.m, t.mInv);
    return t;
}

Xform Xform::LookAt(const float pos[3], const float look[3], const float up[3], bool *ok) {
    float c2w[4][4];
    memset(c2w, 0, sizeof(c2w));
    c2w[0][3] = pos[0];
    c2w[1][3] = pos[1];
    c2w[2][3] = pos[2];
    c2w[3][3] = 1;
    const float lp[3] = {look[0] - pos[0], look[1] - pos[1], look[2] - pos[2]};
    float dir[3], nup[3], left0[3], left[3], newUp[3];
    Normalize3(lp, dir);
    Normalize3(up, nup);
    Cross3(nup, dir, left0);
    if (std::sqrt(left0[0] * left0[0] + left0[1] * left0[1] + left0[2] * left0[2]) == 0) {
        *ok = false;  // transform.cpp:213-219: Error + identity
        return Identity();
    }
    Normalize3(left0, left);
    Cross3(dir, left, newUp);
    for (int k = 0; k < 3; ++k) {
        c2w[k][0] = left[k];
        c2w[k][1] = newUp[k];
        c2w[k][2] = dir[k];
    }
    Xform t;
    memcpy(t.mInv, c2w, sizeof(c2w));
    *ok = MatrixInverse(c2w, t.m);
    return t;
}

Xform Xform::operator*(const Xform &t2) const {
    Xform r;
    MatMul(m, t2.m, r.m);
    MatMul(t2.mInv, mInv, r.mInv);
    return r;
}

Xform Xform::Inverse() const {
    Xform r;
    memcpy(r.m, mInv, sizeof(m));
    memcpy(r.mInv, m, sizeof(m));
    return r;
}

void Xform::ApplyPoint(const float p[3], float out[3]) const {
    const float x = p[0], y = p[1], z = p[2];
    const float xp = m[0][0] * x + m[0][1] * y + m[0][2] * z + m[0][3];
    const float yp = m[1][0] * x + m[1][1] * y + m[1][2] * z + m[1][3];
    const float zp = m[2][0] * x + m[2][1] * y + m[2][2] * z + m[2][3];
    const float wp = m[3][0] * x + m[3][1] * y + m[3][2] * z + m[3][3];
    if (wp == 1) {
        out[0] = xp;
        out[1] = yp;
        out[2] = zp;
    } else {  // Point3 / Float: multiply by 1/wp
        const float inv = 1 / wp;
        out[0] = xp * inv;
        out[1] = yp * inv;
        out[2] = zp * inv;
    }
}

bool Xform::IsIdentity() const {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (m[i][j] != (i == j ? 1.f : 0.f)) return false;
    return true;
}

// ---------------------------------------------------------------------------------------------
// Tokenizer (pbrtlex.ll)

namespace {

struct Token {
    enum Kind { Word, Number, String, LBracket, RBracket, End } kind = End;
    std::string text;
    double num = 0;
    int line = 0;
};

class Lexer {
  public:
    Lexer(std::string text, std::string file) : s_(std::move(text)), file_(std::move(file)) {}
    const std::string &File() const { return file_; }

    Token Next(std::string *err) {
        for (;;) {
            while (pos_ < s_.size() && (s_[pos_] == ' ' || s_[pos_] == '\t' || s_[pos_] == '\r' || s_[pos_] == '\n')) {
                if (s_[pos_] == '\n') ++line_;
                ++pos_;
            }
            if (pos_ < s_.size() && s_[pos_] == '#') {
                while (pos_ < s_.size() && s_[pos_] != '\n') ++pos_;
                continue;
            }
            break;
        }
        Token t;
        t.line = line_;
        if (pos_ >= s_.size()) return t;
        const char c = s_[pos_];
        if (c == '[' || c == ']') {
            t.kind = c == '[' ? Token::LBracket : Token::RBracket;
            ++pos_;
            return t;
        }
        if (c == '"') {
            ++pos_;
            std::string v;
            while (pos_ < s_.size() && s_[pos_] != '"') {
                char ch = s_[pos_++];
                if (ch == '\n') {
                    *err = "unterminated string";
                    return Token();
                }
                if (ch == '\\' && pos_ < s_.size()) {  // pbrtlex.ll escape sequences
                    const char e = s_[pos_++];
                    switch (e) {
                    case 'n': ch = '\n'; break;
                    case 't': ch = '\t'; break;
                    case 'r': ch = '\r'; break;
                    case 'b': ch = '\b'; break;
                    case 'f': ch = '\f'; break;
                    default: ch = e; break;
                    }
                }
                v.push_back(ch);
            }
            if (pos_ >= s_.size()) {
                *err = "unterminated string";
                return Token();
            }
            ++pos_;
            t.kind = Token::String;
            t.text = v;
            return t;
        }
        if ((c >= '0' && c <= '9') || c == '-' || c == '+' || c == '.') {
            const char *b = s_.c_str() + pos_;
            char *e = nullptr;
            t.num = strtod(b, &e);  // atof (pbrtlex.ll:173)
            if (e == b) {
                *err = std::string("illegal character '") + c + "'";
                return Token();
            }
            pos_ += (size_t)(e - b);
            t.kind = Token::Number;
            return t;
        }
        if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_') {
            size_t b = pos_;
            while (pos_ < s_.size() && (isalnum((unsigned char)s_[pos_]) || s_[pos_] == '_')) ++pos_;
            t.kind = Token::Word;
            t.text = s_.substr(b, pos_ - b);
            return t;
        }
        *err = std::string("illegal character '") + c + "'";
        return Token();
    }

    Token Peek(std::string *err) {
        const size_t p = pos_;
        const int l = line_;
        Token t = Next(err);
        pos_ = p;
        line_ = l;
        return t;
    }

  private:
    std::string s_;
    std::string file_;
    size_t pos_ = 0;
    int line_ = 1;
};

// pbrtparse.y lookupType: "type name" -> canonical type
bool LookupType(const std::string &decl, std::string *type, std::string *name) {
    std::istringstream is(decl);
    std::string t, n, extra;
    if (!(is >> t >> n) || (is >> extra)) return false;
    if (t == "point") t = "point3";
    if (t == "vector") t = "vector3";
    if (t == "normal") t = "normal3";
    if (t == "color") t = "rgb";
    static const char *known[] = {"integer", "float", "point2", "vector2", "point3", "vector3", "normal3",
                                  "rgb", "xyz", "blackbody", "spectrum", "bool", "string", "texture"};
    bool ok = false;
    for (const char *k : known) ok = ok || t == k;
    if (!ok) return false;
    *type = t;
    *name = n;
    return true;
}

struct Material {
    std::string type = "matte";
    float kd[3] = {0.5f, 0.5f, 0.5f};  // MatteMaterial "Kd" default 0.5 (materials/matte.cpp)
    float sigma = 0.f;
    bool none = false;
};

struct GraphicsState {
    Material material;
    std::string namedMaterial;
    std::string inside, outside;
    bool areaLight = false;
    float areaL[3] = {1, 1, 1};
    bool reverseOrientation = false;
};

struct MediumDef {
    int kind = BRE_MEDIUM_NONE;
    float sigma_a[3], sigma_s[3], g = 0;
    int n[3] = {1, 1, 1};
    std::vector<float> density;
    float worldToMedium[4][4];
};

struct ShapeRec {
    bre_triangle tri;
    std::string inside, outside;
};

class Parser {
  public:
    explicit Parser(PbrtScene *out) : out_(out) {}

    bool Run(Lexer &lx, int depth);
    bool Finish();

  private:
    void Error(const Lexer &lx, int line, const char *fmt, ...);
    void Warning(const Lexer &lx, int line, const char *fmt, ...);
    bool ReadParams(Lexer &lx, ParamSet *ps, std::string *err);
    bool ReadNumbers(Lexer &lx, int n, double *v, std::string *err);
    bool ReadNumArray(Lexer &lx, std::vector<double> *v, std::string *err);
    void ReportUnused(const Lexer &lx, int line, const ParamSet &ps);
    void Shape(Lexer &lx, int line, const std::string &name, const ParamSet &ps);
    void MakeMedium(Lexer &lx, int line, const std::string &name, const ParamSet &ps);
    void MakeMaterial(Lexer &lx, int line, const std::string &type, const ParamSet &ps, Material *m);
    void Camera(Lexer &lx, int line, const std::string &name, const ParamSet &ps);
    void Concat(const Xform &t) {
        ctm_ = ctm_ * t;
        ctmKind_ = 2;
    }

    PbrtScene *out_;
    Xform ctm_ = Xform::Identity();
    int ctmKind_ = 0;  // 0 identity, 1 exactly one LookAt, 2 anything else
    float lookAt_[9] = {0, 0, 0, 0, 0, 1, 0, 1, 0};
    std::vector<std::pair<Xform, int>> xformStack_;
    std::vector<std::array<float, 9>> lookStack_;
    GraphicsState gs_;
    std::vector<GraphicsState> gsStack_;
    std::map<std::string, Xform> coordSys_;
    std::map<std::string, MediumDef> media_;
    std::map<std::string, Material> namedMaterials_;
    std::vector<ShapeRec> shapes_;
    bool inWorld_ = false, worldEnded_ = false;
    bool cameraLookAtOk_ = false;
    float camLook_[9];
    float camFov_ = 90.f;
};

// ---------------------------------------------------------------------------------------------
// Parser (pbrtparse.y + api.cpp)

void Parser::Error(const Lexer &lx, int line, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    out_->messages += "Error: " + lx.File() + "(" + std::to_string(line) + "): " + buf + "\n";
    ++out_->errors;
}

void Parser::Warning(const Lexer &lx, int line, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    out_->messages += "Warning: " + lx.File() + "(" + std::to_string(line) + "): " + buf + "\n";
    ++out_->warnings;
}

bool Parser::ReadNumbers(Lexer &lx, int n, double *v, std::string *err) {
    for (int i = 0; i < n; ++i) {
        Token t = lx.Next(err);
        if (t.kind != Token::Number) {
            if (err->empty()) *err = "expected a number";
            return false;
        }
        v[i] = t.num;
    }
    return true;
}

bool Parser::ReadNumArray(Lexer &lx, std::vector<double> *v, std::string *err) {
    Token t = lx.Next(err);
    if (t.kind == Token::Number) {
        v->push_back(t.num);
        return true;
    }
    if (t.kind != Token::LBracket) {
        if (err->empty()) *err = "expected '[' or a number";
        return false;
    }
    for (;;) {
        t = lx.Next(err);
        if (t.kind == Token::RBracket) return true;
        if (t.kind != Token::Number) {
            if (err->empty()) *err = "expected a number or ']'";
            return false;
        }
        v->push_back(t.num);
    }
}

// paramlist: ("type name" value | "type name" [ values ])*
bool Parser::ReadParams(Lexer &lx, ParamSet *ps, std::string *err) {
    for (;;) {
        Token t = lx.Peek(err);
        if (!err->empty()) return false;
        if (t.kind != Token::String) return true;
        lx.Next(err);
        ParamItem it;
        const bool typed = LookupType(t.text, &it.type, &it.name);
        std::vector<double> nums;
        std::vector<std::string> strs;
        Token v = lx.Next(err);
        auto take = [&](const Token &x) -> bool {
            if (x.kind == Token::Number) nums.push_back(x.num);
            else if (x.kind == Token::String) strs.push_back(x.text);
            else return false;
            return true;
        };
        if (v.kind == Token::LBracket) {
            for (;;) {
                Token x = lx.Next(err);
                if (x.kind == Token::RBracket) break;
                if (!take(x)) {
                    if (err->empty()) *err = "bad value in parameter list of \"" + t.text + "\"";
                    return false;
                }
            }
        } else if (!take(v)) {
            if (err->empty()) *err = "missing value for parameter \"" + t.text + "\"";
            return false;
        }
        if (!nums.empty() && !strs.empty()) {
            *err = "mixed string and numeric values for \"" + t.text + "\"";
            return false;
        }
        if (!typed) {
            Error(lx, t.line, "Unable to decode type for name \"%s\"", t.text.c_str());
            continue;
        }
        const std::string &ty = it.type;
        if (ty == "string" || ty == "texture") {
            if (!nums.empty()) {
                Error(lx, t.line, "Expected string parameter value for parameter \"%s\"", it.name.c_str());
                continue;
            }
            it.strings = strs;
        } else if (ty == "bool") {
            bool ok = nums.empty();
            for (auto &s : strs) {
                if (s == "true") it.bools.push_back(true);
                else if (s == "false") it.bools.push_back(false);
                else ok = false;
            }
            if (!ok) {
                Error(lx, t.line, "Value for \"%s\" must be \"true\" or \"false\"", it.name.c_str());
                continue;
            }
        } else {
            if (!strs.empty()) {
                Error(lx, t.line, "Expected numeric parameter value for parameter \"%s\"", it.name.c_str());
                continue;
            }
            if (ty == "integer") {
                for (double d : nums) {
                    if ((double)(int)d != d)
                        Warning(lx, t.line, "Floating-point value provided for integer parameter \"%s\"", it.name.c_str());
                    it.ints.push_back((int)d);  // pbrtparse.y: ints converted from the doubles
                }
            } else {
                for (double d : nums) it.floats.push_back((float)d);
                int per = 1;
                if (ty == "point2" || ty == "vector2") per = 2;
                if (ty == "point3" || ty == "vector3" || ty == "normal3" || ty == "rgb" || ty == "xyz") per = 3;
                if (it.floats.size() % per != 0) {
                    Error(lx, t.line, "Excess values given with \"%s\" parameter \"%s\"", ty.c_str(), it.name.c_str());
                    continue;
                }
            }
        }
        ps->Add(std::move(it));
    }
}

void Parser::ReportUnused(const Lexer &lx, int line, const ParamSet &ps) {
    for (auto &u : ps.Unused()) Warning(lx, line, "Parameter %s not used", u.c_str());
}

void Parser::Camera(Lexer &lx, int line, const std::string &name, const ParamSet &ps) {
    out_->cameraName = name;
    if (name != "perspective") {
        Error(lx, line, "Camera \"%s\" is not supported by the GPU camera pass (perspective only)", name.c_str());
        return;
    }
    if (ctmKind_ == 2) {
        Error(lx, line, "Camera: the CTM must be Identity followed by at most one LookAt (the GPU camera is built "
                        "from LookAt eye/look/up)");
        return;
    }
    // perspective.cpp:236-275
    float fov = ps.FindOneFloat("fov", 90.f);
    const float halffov = ps.FindOneFloat("halffov", -1.f);
    if (halffov > 0.f) fov = 2.f * halffov;
    if (ps.FindOneFloat("lensradius", 0.f) != 0.f) {
        Error(lx, line, "Camera: \"lensradius\" must be 0 (pinhole only)");
        return;
    }
    ps.FindOneFloat("focaldistance", 1e6f);
    ps.FindOneFloat("shutteropen", 0.f);
    ps.FindOneFloat("shutterclose", 1.f);
    if (ps.Has("screenwindow") || ps.Has("frameaspectratio")) {
        Error(lx, line, "Camera: \"screenwindow\" / \"frameaspectratio\" are not supported");
        return;
    }
    ReportUnused(lx, line, ps);
    memcpy(camLook_, lookAt_, sizeof(camLook_));
    camFov_ = fov;
    out_->haveCamera = true;
}

void Parser::MakeMaterial(Lexer &lx, int line, const std::string &type, const ParamSet &ps, Material *m) {
    *m = Material();
    m->type = type;
    if (type == "" || type == "none") {
        m->none = true;
        return;
    }
    if (type != "matte") {
        Error(lx, line, "Material \"%s\" is not supported (matte only); using \"matte\"", type.c_str());
        m->type = "matte";
    }
    if (ps.Has("Kd") && !ps.FindOneSpectrum("Kd", m->kd))
        Error(lx, line, "matte \"Kd\" must be an rgb or xyz value (textures are not supported)");
    m->sigma = ps.FindOneFloat("sigma", 0.f);
    if (m->sigma != 0.f) Error(lx, line, "matte \"sigma\" must be 0 (Oren-Nayar is not supported)");
    ps.FindOneString("type", "");
    ReportUnused(lx, line, ps);
}

void Parser::MakeMedium(Lexer &lx, int line, const std::string &name, const ParamSet &ps) {
    const std::string type = ps.FindOneString("type", "");
    if (type.empty()) {
        Error(lx, line, "No parameter string \"type\" found in MakeNamedMedium");
        return;
    }
    // api.cpp:547-593
    MediumDef m;
    float sa[3] = {.0011f, .0024f, .014f}, ss[3] = {2.55f, 3.21f, 3.77f};
    const std::string preset = ps.FindOneString("preset", "");
    if (!preset.empty()) Warning(lx, line, "Material preset \"%s\" not found.  Using defaults.", preset.c_str());
    const float scale = ps.FindOneFloat("scale", 1.f);
    m.g = ps.FindOneFloat("g", 0.0f);
    ps.FindOneSpectrum("sigma_a", sa);
    ps.FindOneSpectrum("sigma_s", ss);
    for (int k = 0; k < 3; ++k) {
        m.sigma_a[k] = sa[k] * scale;
        m.sigma_s[k] = ss[k] * scale;
    }
    if (type == "homogeneous") {
        m.kind = BRE_MEDIUM_HOMOGENEOUS;
        MatIdentity(m.worldToMedium);
    } else if (type == "heterogeneous") {
        const std::vector<float> *data = ps.FindFloats("density");
        if (!data) {
            Error(lx, line, "No \"density\" values provided for heterogeneous medium?");
            return;
        }
        m.n[0] = ps.FindOneInt("nx", 1);
        m.n[1] = ps.FindOneInt("ny", 1);
        m.n[2] = ps.FindOneInt("nz", 1);
        float p0[3] = {0, 0, 0}, p1[3] = {1, 1, 1};
        ps.FindOnePoint3f("p0", p0);
        ps.FindOnePoint3f("p1", p1);
        if ((int64_t)data->size() != (int64_t)m.n[0] * m.n[1] * m.n[2]) {
            Error(lx, line, "GridDensityMedium has %d density values; expected nx*ny*nz = %d", (int)data->size(),
                  m.n[0] * m.n[1] * m.n[2]);
            return;
        }
        m.kind = BRE_MEDIUM_GRID;
        m.density = *data;
        // WorldToMedium = Inverse(medium2world * Translate(p0) * Scale(p1 - p0)) (grid.h:58)
        const Xform d2m = Xform::Translate(p0[0], p0[1], p0[2]) * Xform::Scale(p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]);
        const Xform m2w = ctm_ * d2m;
        memcpy(m.worldToMedium, m2w.mInv, sizeof(m.worldToMedium));
    } else {
        Warning(lx, line, "Medium \"%s\" unknown.", type.c_str());
        return;
    }
    ReportUnused(lx, line, ps);
    media_[name] = std::move(m);
}

void Parser::Shape(Lexer &lx, int line, const std::string &name, const ParamSet &ps) {
    if (name != "trianglemesh") {
        Error(lx, line, "Shape \"%s\" is not supported (\"trianglemesh\" only)", name.c_str());
        return;
    }
    const std::vector<int> *idx = ps.FindInts("indices");
    const std::vector<float> *P = ps.FindPoint3fs("P");
    if (!idx || !P) {
        Error(lx, line, "trianglemesh needs \"integer indices\" and \"point P\"");
        return;
    }
    for (const char *n : {"uv", "st", "N", "S", "alpha", "shadowalpha", "faceIndices"})
        if (ps.Has(n)) Warning(lx, line, "trianglemesh \"%s\" is ignored by the GPU scene model", n);
    const size_t nv = P->size() / 3;
    // CreateTriangleMeshShape (shapes/triangle.cpp): indices in triples
    if (idx->size() % 3 != 0) {
        Error(lx, line, "Number of vertex indices %d not a multiple of 3", (int)idx->size());
        return;
    }
    for (int i : *idx)
        if (i < 0 || (size_t)i >= nv) {
            Error(lx, line, "trianglemesh has out of-bounds vertex index %d (%d \"P\" values were given)", i, (int)nv);
            return;
        }
    Material mat = gs_.material;
    if (!gs_.namedMaterial.empty()) {
        auto it = namedMaterials_.find(gs_.namedMaterial);
        if (it != namedMaterials_.end()) mat = it->second;
        else {
            Error(lx, line, "Named material \"%s\" not defined. Using \"matte\".", gs_.namedMaterial.c_str());
            mat = Material();
        }
    }
    if (mat.none) {
        Error(lx, line, "shapes without a material (medium boundaries) are not supported by the GPU scene model");
        return;
    }
    // vertices to world space as TriangleMesh does (mesh->p[i] = ObjectToWorld(P[i]))
    std::vector<float> W(P->size());
    for (size_t v = 0; v < nv; ++v) ctm_.ApplyPoint(&(*P)[3 * v], &W[3 * v]);
    // Triangle::reverseOrientation ^ transformSwapsHandedness (Transform::SwapsHandedness: the
    // determinant of the upper-left 3x3 is negative, transform.cpp)
    float det = 0.f;
    {
        const float (*m)[4] = ctm_.m;
        det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
              m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    }
    const bool flip = gs_.reverseOrientation != (det < 0);
    for (size_t t = 0; t < idx->size() / 3; ++t) {
        ShapeRec sr;
        memset(&sr.tri, 0, sizeof(sr.tri));
        for (int v = 0; v < 3; ++v) memcpy(sr.tri.p[v], &W[3 * (*idx)[3 * t + v]], 3 * sizeof(float));
        memcpy(sr.tri.kd, mat.kd, sizeof(sr.tri.kd));
        sr.tri.flip = flip ? 1 : 0;
        if (gs_.areaLight) {
            // pbrtShape: one DiffuseAreaLight per shape of the mesh (api.cpp), one-sided
            sr.tri.emit = 1;
            memcpy(sr.tri.Le, gs_.areaL, sizeof(sr.tri.Le));
        }
        sr.inside = gs_.inside;
        sr.outside = gs_.outside;
        shapes_.push_back(sr);
    }
    ReportUnused(lx, line, ps);
}

bool Parser::Run(Lexer &lx, int depth) {
    std::string err;
    for (;;) {
        Token t = lx.Next(&err);
        if (!err.empty()) break;
        if (t.kind == Token::End) return true;
        const int line = t.line;
        if (t.kind != Token::Word) {
            err = "syntax error: expected a directive";
            break;
        }
        const std::string &w = t.text;
        auto str = [&](std::string *s) -> bool {
            Token x = lx.Next(&err);
            if (x.kind != Token::String) {
                if (err.empty()) err = "expected a quoted string after " + w;
                return false;
            }
            *s = x.text;
            return true;
        };
        if (worldEnded_) {
            Warning(lx, line, "%s after WorldEnd ignored", w.c_str());
        }
        if (w == "Identity") {
            ctm_ = Xform::Identity();
            ctmKind_ = 0;
        } else if (w == "Translate" || w == "Scale") {
            double v[3];
            if (!ReadNumbers(lx, 3, v, &err)) break;
            Concat(w == "Translate" ? Xform::Translate((float)v[0], (float)v[1], (float)v[2])
                                    : Xform::Scale((float)v[0], (float)v[1], (float)v[2]));
        } else if (w == "Rotate") {
            double v[4];
            if (!ReadNumbers(lx, 4, v, &err)) break;
            Concat(Xform::Rotate((float)v[0], (float)v[1], (float)v[2], (float)v[3]));
        } else if (w == "LookAt") {
            double v[9];
            if (!ReadNumbers(lx, 9, v, &err)) break;
            float f[9];
            for (int k = 0; k < 9; ++k) f[k] = (float)v[k];
            bool ok = true;
            const Xform la = Xform::LookAt(f, f + 3, f + 6, &ok);
            if (!ok)
                Error(lx, line, "\"up\" vector and viewing direction passed to LookAt are pointing in the same "
                                "direction.  Using the identity transformation.");
            const int kind = ctmKind_;
            ctm_ = ctm_ * la;
            if (kind == 0 && ok) {
                ctmKind_ = 1;
                memcpy(lookAt_, f, sizeof(f));
            } else if (ok) {
                ctmKind_ = 2;
            }
        } else if (w == "Transform" || w == "ConcatTransform") {
            std::vector<double> v;
            if (!ReadNumArray(lx, &v, &err)) break;
            if (v.size() != 16) {
                Error(lx, line, "%s needs 16 values", w.c_str());
                continue;
            }
            float rm[4][4];  // pbrtTransform: the file is column-major
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) rm[i][j] = (float)v[4 * j + i];
            const Xform x = Xform::FromMatrix(rm);
            if (w == "Transform") {
                ctm_ = x;
                ctmKind_ = 2;
            } else {
                Concat(x);
            }
        } else if (w == "CoordinateSystem") {
            std::string n;
            if (!str(&n)) break;
            coordSys_[n] = ctm_;
        } else if (w == "CoordSysTransform") {
            std::string n;
            if (!str(&n)) break;
            auto it = coordSys_.find(n);
            if (it != coordSys_.end()) {
                ctm_ = it->second;
                ctmKind_ = 2;
            } else {
                Warning(lx, line, "Couldn't find named coordinate system \"%s\"", n.c_str());
            }
        } else if (w == "ActiveTransform") {
            Token x = lx.Next(&err);
            if (x.kind != Token::Word) {
                if (err.empty()) err = "ActiveTransform needs StartTime, EndTime or All";
                break;
            }
            Warning(lx, line, "ActiveTransform ignored (no motion blur)");
        } else if (w == "TransformTimes") {
            double v[2];
            if (!ReadNumbers(lx, 2, v, &err)) break;
        } else if (w == "ReverseOrientation") {
            gs_.reverseOrientation = !gs_.reverseOrientation;
        } else if (w == "WorldBegin") {
            inWorld_ = true;
            ctm_ = Xform::Identity();
            ctmKind_ = 0;
            coordSys_["world"] = ctm_;
        } else if (w == "WorldEnd") {
            worldEnded_ = true;
        } else if (w == "AttributeBegin" || w == "TransformBegin") {
            xformStack_.push_back({ctm_, ctmKind_});
            std::array<float, 9> la;
            memcpy(la.data(), lookAt_, sizeof(lookAt_));
            lookStack_.push_back(la);
            if (w == "AttributeBegin") gsStack_.push_back(gs_);
        } else if (w == "AttributeEnd" || w == "TransformEnd") {
            if (w == "AttributeEnd") {
                if (gsStack_.empty()) {
                    Error(lx, line, "Unmatched pbrtAttributeEnd() encountered. Ignoring it.");
                    continue;
                }
                gs_ = gsStack_.back();
                gsStack_.pop_back();
            }
            if (xformStack_.empty()) {
                Error(lx, line, "Unmatched %s encountered. Ignoring it.", w.c_str());
                continue;
            }
            ctm_ = xformStack_.back().first;
            ctmKind_ = xformStack_.back().second;
            memcpy(lookAt_, lookStack_.back().data(), sizeof(lookAt_));
            xformStack_.pop_back();
            lookStack_.pop_back();
        } else if (w == "Include") {
            std::string f;
            if (!str(&f)) break;
            if (depth > 16) {
                err = "Include nested too deeply";
                break;
            }
            std::string path = f;
            const size_t slash = lx.File().find_last_of('/');
            if (!f.empty() && f[0] != '/' && slash != std::string::npos) path = lx.File().substr(0, slash + 1) + f;
            std::ifstream in(path, std::ios::binary);
            if (!in) {
                Error(lx, line, "Unable to open included file \"%s\"", path.c_str());
                continue;
            }
            std::stringstream ss;
            ss << in.rdbuf();
            Lexer sub(ss.str(), path);
            if (!Run(sub, depth + 1)) return false;
        } else if (w == "MediumInterface") {
            std::string a, b;
            if (!str(&a)) break;
            Token x = lx.Peek(&err);
            if (x.kind == Token::String) {
                str(&b);
            } else {
                b = a;  // pbrtparse.y: a single name is both inside and outside
            }
            gs_.inside = a;
            gs_.outside = b;
        } else if (w == "NamedMaterial") {
            std::string n;
            if (!str(&n)) break;
            gs_.namedMaterial = n;
        } else if (w == "ObjectBegin" || w == "ObjectInstance") {
            std::string n;
            if (!str(&n)) break;
            Error(lx, line, "%s is not supported by the GPU scene model", w.c_str());
        } else if (w == "ObjectEnd") {
        } else if (w == "Camera" || w == "Film" || w == "Sampler" || w == "PixelFilter" || w == "Accelerator" ||
                   w == "Integrator" || w == "Shape" || w == "Material" || w == "LightSource" ||
                   w == "AreaLightSource" || w == "MakeNamedMedium" || w == "MakeNamedMaterial" || w == "Texture") {
            std::string n, n2, n3;
            if (!str(&n)) break;
            if (w == "Texture") {
                if (!str(&n2) || !str(&n3)) break;
            }
            ParamSet ps;
            if (!ReadParams(lx, &ps, &err)) break;
            if (w == "Camera") {
                if (inWorld_) Error(lx, line, "Camera must be set before WorldBegin");
                else Camera(lx, line, n, ps);
            } else if (w == "Film") {
                if (n != "image") Warning(lx, line, "Film \"%s\" unknown; using \"image\"", n.c_str());
                FilmDesc &f = out_->film;
                f.xres = ps.FindOneInt("xresolution", 1280);
                f.yres = ps.FindOneInt("yresolution", 720);
                const std::string fn = ps.FindOneString("filename", "");
                f.filename = fn.empty() ? "pbrt.pfm" : fn;
                f.scale = ps.FindOneFloat("scale", 1.f);
                ps.FindOneFloat("diagonal", 35.f);
                ps.FindOneFloat("maxsampleluminance", INFINITY);
                if (ps.Has("cropwindow") || ps.Has("pixelbounds"))
                    Error(lx, line, "Film \"cropwindow\" / \"pixelbounds\" are not supported");
                ReportUnused(lx, line, ps);
            } else if (w == "Sampler" || w == "PixelFilter" || w == "Accelerator") {
                // the photon-beam integrator uses neither (see pbrt_scene.h)
            } else if (w == "Integrator") {
                out_->integratorName = n;
                out_->integratorParams = ps;
            } else if (w == "Shape") {
                if (!inWorld_) Error(lx, line, "Shape not allowed outside WorldBegin/WorldEnd");
                else Shape(lx, line, n, ps);
            } else if (w == "Material") {
                MakeMaterial(lx, line, n, ps, &gs_.material);
                gs_.namedMaterial.clear();
            } else if (w == "MakeNamedMaterial") {
                const std::string type = ps.FindOneString("type", "");
                if (type.empty()) {
                    Error(lx, line, "No parameter string \"type\" found in MakeNamedMaterial");
                } else {
                    Material m;
                    MakeMaterial(lx, line, type, ps, &m);
                    namedMaterials_[n] = m;
                }
            } else if (w == "LightSource") {
                Error(lx, line, "LightSource \"%s\" is not supported (diffuse area lights only)", n.c_str());
            } else if (w == "AreaLightSource") {
                if (n != "diffuse" && n != "area") {
                    Error(lx, line, "AreaLightSource \"%s\" unknown", n.c_str());
                } else {
                    // lights/diffuse.cpp:136-150: L * scale, one-sided
                    float L[3] = {1, 1, 1}, sc[3] = {1, 1, 1};
                    ps.FindOneSpectrum("L", L);
                    ps.FindOneSpectrum("scale", sc);
                    ps.FindOneInt("samples", ps.FindOneInt("nsamples", 1));
                    if (ps.FindOneBool("twosided", false))
                        Error(lx, line, "two-sided area lights are not supported");
                    for (int k = 0; k < 3; ++k) gs_.areaL[k] = L[k] * sc[k];
                    gs_.areaLight = true;
                    ReportUnused(lx, line, ps);
                }
            } else if (w == "MakeNamedMedium") {
                MakeMedium(lx, line, n, ps);
            } else if (w == "Texture") {
                Error(lx, line, "textures are not supported by the GPU scene model");
            }
        } else {
            err = "unknown directive \"" + w + "\"";
            break;
        }
    }
    out_->messages += "Error: " + lx.File() + ": " + err + "\n";
    ++out_->errors;
    return false;
}

bool Parser::Finish() {
    PbrtScene &o = *out_;
    auto fatal = [&](const std::string &m) {
        o.messages += "Error: " + m + "\n";
        ++o.errors;
        return false;
    };
    if (!o.haveCamera) return fatal("no usable perspective Camera");
    if (shapes_.empty()) return fatal("the scene has no shapes");
    if ((int64_t)shapes_.size() > BRE_MAX_SCENE_TRIANGLES)
        return fatal("more than BRE_MAX_SCENE_TRIANGLES (" + std::to_string(BRE_MAX_SCENE_TRIANGLES) + ") triangles");
    int nemit = 0;
    for (size_t i = 0; i < shapes_.size(); ++i) nemit += shapes_[i].tri.emit != 0;
    if (nemit == 0) return fatal("the scene has no diffuse area light");
    // The camera medium is the outside medium of the graphics state at WorldEnd (api.cpp:651-655).
    const std::string M = gs_.outside;
    const MediumDef *med = nullptr;
    if (!M.empty()) {
        auto it = media_.find(M);
        if (it == media_.end()) return fatal("Named medium \"" + M + "\" undefined.");
        med = &it->second;
    }
    // One medium fills all space: a non-transition interface ("" "") keeps the ray's medium
    // (GeometricPrimitive::Intersect), an (M, M) interface re-enters M; photons leave the light
    // through its own interface, so the emitter must carry (M, M) when M is not vacuum.
    for (size_t i = 0; i < shapes_.size(); ++i) {
        const ShapeRec &s = shapes_[i];
        const bool inherit = s.inside.empty() && s.outside.empty();
        const bool same = s.inside == M && s.outside == M;
        if (s.tri.emit ? !same : !(inherit || same))
            return fatal("shape " + std::to_string(i) + " has MediumInterface \"" + s.inside + "\" \"" + s.outside +
                         "\"; the GPU scene model has one medium (\"" + M + "\") filling all space");
    }
    bre_scene &sc = o.scene;
    memset(&sc, 0, sizeof(sc));
    sc.n_triangles = (int32_t)shapes_.size();
    // up to BRE_MAX_TRIANGLES inline, any number through triangles_ext (PbrtScene::triangles)
    if (shapes_.size() <= (size_t)BRE_MAX_TRIANGLES) {
        for (size_t i = 0; i < shapes_.size(); ++i) sc.triangles[i] = shapes_[i].tri;
    } else {
        o.triangles.resize(shapes_.size());
        for (size_t i = 0; i < shapes_.size(); ++i) o.triangles[i] = shapes_[i].tri;
    }
    if (med) {
        sc.has_medium = med->kind;
        memcpy(sc.sigma_a, med->sigma_a, sizeof(sc.sigma_a));
        memcpy(sc.sigma_s, med->sigma_s, sizeof(sc.sigma_s));
        sc.g = med->g;
        if (med->kind == BRE_MEDIUM_GRID) {
            memcpy(sc.grid_n, med->n, sizeof(sc.grid_n));
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) sc.world_to_medium[4 * i + j] = med->worldToMedium[i][j];
            o.density = med->density;
        }
    }
    memcpy(sc.cam_pos, camLook_, 12);
    memcpy(sc.cam_look, camLook_ + 3, 12);
    memcpy(sc.cam_up, camLook_ + 6, 12);
    sc.cam_fov_deg = camFov_;
    o.Bind();
    if (o.integratorName.empty()) o.integratorName = "path";  // pbrt's default integrator
    return true;
}

}  // namespace

void PbrtScene::Bind() {
    scene.grid_density = density.empty() ? nullptr : density.data();
    scene.triangles_ext = triangles.empty() ? nullptr : triangles.data();
}

static bool ParseLexer(Lexer &lx, PbrtScene *out) {
    *out = PbrtScene();
    Parser p(out);
    if (!p.Run(lx, 0)) return false;
    return p.Finish();
}

bool ParsePbrtFile(const std::string &path, PbrtScene *out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        *out = PbrtScene();
        out->messages = "Error: Couldn't open scene file \"" + path + "\"\n";
        out->errors = 1;
        return false;
    }
    std::stringstream ss;
    ss << in.rdbuf();
    Lexer lx(ss.str(), path);
    return ParseLexer(lx, out);
}

bool ParsePbrtString(const std::string &text, PbrtScene *out) {
    Lexer lx(text, "<string>");
    return ParseLexer(lx, out);
}

// ---------------------------------------------------------------------------------------------
// Film and PFM (film.cpp:132-210, imageio.cpp:437-482)

void FilmFinalize(const float *L, int64_t npix, float scale, float *out) {
    for (int64_t i = 0; i < npix; ++i) {
        const float *c = L + 3 * i;
        // Film::SetImage: RGBSpectrum::ToXYZ = RGBToXYZ (spectrum.h:62-66); filterWeightSum = 1
        float xyz[3];
        xyz[0] = 0.412453f * c[0] + 0.357580f * c[1] + 0.180423f * c[2];
        xyz[1] = 0.212671f * c[0] + 0.715160f * c[1] + 0.072169f * c[2];
        xyz[2] = 0.019334f * c[0] + 0.119193f * c[1] + 0.950227f * c[2];
        // Film::WriteImage: XYZToRGB, * (1 / filterWeightSum), max(0, .)
        float rgb[3];
        rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
        rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
        rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
        const float invWt = (float)1 / 1.f;
        for (int k = 0; k < 3; ++k) {
            float v = std::max(0.f, rgb[k] * invWt);
            v += 1.f * 0.f;  // splatScale * splatRGB: SetImage zeroes the splats
            out[3 * i + k] = v * scale;
        }
    }
}

bool WritePFM(const std::string &filename, const float *rgb, int width, int height, std::string *err) {
    FILE *fp = fopen(filename.c_str(), "wb");
    if (!fp) {
        if (err) *err = "Unable to open output PFM file \"" + filename + "\"";
        return false;
    }
    bool ok = fprintf(fp, "PF\n") >= 0 && fprintf(fp, "%d %d\n", width, height) >= 0 &&
              fprintf(fp, "%f\n", -1.f) >= 0;  // negative scale: little endian (x86-64 and gfx hosts)
    for (int y = height - 1; ok && y >= 0; y--)  // rows bottom to top
        ok = fwrite(rgb + (size_t)y * width * 3, sizeof(float), (size_t)width * 3, fp) == (size_t)width * 3;
    if (fclose(fp) != 0) ok = false;
    if (!ok && err) *err = "Error writing PFM file \"" + filename + "\"";
    return ok;
}

bool ReadPFM(const std::string &filename, std::vector<float> *rgb, int *width, int *height, std::string *err) {
    FILE *fp = fopen(filename.c_str(), "rb");
    if (!fp) {
        if (err) *err = "Error reading PFM file \"" + filename + "\"";
        return false;
    }
    char magic[3] = {0, 0, 0};
    int w = 0, h = 0;
    float scale = 0;
    bool ok = fscanf(fp, "%2s", magic) == 1 && (magic[0] == 'P' && (magic[1] == 'F' || magic[1] == 'f')) &&
              fscanf(fp, "%d %d", &w, &h) == 2 && w > 0 && h > 0 && fscanf(fp, "%f", &scale) == 1 && fgetc(fp) != EOF;
    const int nch = magic[1] == 'F' ? 3 : 1;
    std::vector<float> data;
    if (ok) {
        data.resize((size_t)w * h * nch);
        ok = fread(data.data(), sizeof(float), data.size(), fp) == data.size();
    }
    fclose(fp);
    if (!ok || scale >= 0.f) {  // big-endian PFMs are not produced on any host this runs on
        if (err) *err = "Error reading PFM file \"" + filename + "\"";
        return false;
    }
    const float absScale = std::fabs(scale);
    rgb->assign((size_t)w * h * 3, 0.f);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            for (int k = 0; k < 3; ++k) {
                float v = data[((size_t)y * w + x) * nch + (nch == 3 ? k : 0)];
                if (absScale != 1.f) v *= absScale;
                (*rgb)[((size_t)(h - 1 - y) * w + x) * 3 + k] = v;  // flip to top-row first
            }
    *width = w;
    *height = h;
    return true;
}

}  // namespace bre_host
