// mof_ply.cpp -- SURVEY.md §8(f)3: the S3 surface without pyvista / VTK.
//
// S3 reads the cortical surface with pyvista (S3…py:75-84):
//   coordinates = surface.points                       (float32, VTK points)
//   triangles   = surface.faces.reshape(-1, 4)[:, 1:]  (all-triangle mesh)
//   normals     = surface.point_normals                (vtkPolyDataNormals)
//   areas       = surface.compute_cell_sizes(...)['Area']  (vtkCellSizeFilter)
// VTK is not installed in this image, so these restate the published VTK
// algorithms (parity unpinned: no VTK output to check against):
//  * PLY: ascii / binary_little_endian / binary_big_endian; element vertex
//    with x, y, z (any scalar type, stored as float32 like vtkPLYReader) and
//    optional nx, ny, nz; element face with a list property vertex_indices
//    (or vertex_index); other elements and properties are skipped;
//  * point normals (vtkPolyDataNormals as pyvista's compute_normals calls it:
//    no splitting, consistent input ordering assumed, no auto-orientation):
//    per triangle n = (p2 - p1) x (p0 - p1), normalised, in double from the
//    float32 points; per point the sum of its triangles' normals in triangle
//    order, normalised, stored as float32;
//  * cell areas: 0.5 |(p1 - p0) x (p2 - p0)| in double.
// A PLY that carries nx, ny, nz gives those normals (pyvista returns the
// file's "Normals" array when present).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

#include "mof_internal.h"

int mof_io_guard(const std::function<void()> &f);  // mof_abi.cpp

namespace mof {
namespace {

enum class Fmt { Ascii, BinLE, BinBE };

struct Prop {
    std::string name, type, count_type;  // count_type non-empty for lists
    bool list() const { return !count_type.empty(); }
};

struct Elem {
    std::string name;
    int64_t count = 0;
    std::vector<Prop> props;
};

int type_size(const std::string &t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    throw Error{MOF_E_ARG, "PLY: unknown property type " + t};
}

struct Ply {
    Fmt fmt = Fmt::Ascii;
    std::vector<Elem> elems;
    std::vector<char> body;  // everything after end_header
};

Ply parse_header(const char *path) {
    std::ifstream f(path, std::ios::binary);
    MOF_REQUIRE(f.good(), std::string("cannot open ") + path);
    Ply ply;
    std::string line;
    std::getline(f, line);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    MOF_REQUIRE(line == "ply", "not a PLY file");
    bool ended = false;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string kw;
        ss >> kw;
        if (kw == "format") {
            std::string fm;
            ss >> fm;
            if (fm == "ascii") ply.fmt = Fmt::Ascii;
            else if (fm == "binary_little_endian") ply.fmt = Fmt::BinLE;
            else if (fm == "binary_big_endian") ply.fmt = Fmt::BinBE;
            else throw Error{MOF_E_ARG, "PLY: unknown format " + fm};
        } else if (kw == "element") {
            Elem e;
            ss >> e.name >> e.count;
            MOF_REQUIRE(!ss.fail() && e.count >= 0, "PLY: bad element count");
            for (const Elem &o : ply.elems)
                MOF_REQUIRE(o.name != e.name, "PLY: duplicate element " + e.name);
            ply.elems.push_back(e);
        } else if (kw == "property") {
            MOF_REQUIRE(!ply.elems.empty(), "PLY: property before element");
            Prop p;
            std::string t;
            ss >> t;
            if (t == "list") {
                ss >> p.count_type >> p.type >> p.name;
                (void)type_size(p.count_type);
            } else {
                p.type = t;
                ss >> p.name;
            }
            (void)type_size(p.type);  // unknown types are rejected here
            ply.elems.back().props.push_back(p);
        } else if (kw == "end_header") {
            ended = true;
            break;
        }
    }
    MOF_REQUIRE(ended, "PLY: no end_header");
    ply.body.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    // every record needs at least one byte per value (ascii: a digit; binary:
    // the scalar / list-count sizes): element counts the body cannot hold
    // are rejected before anything is allocated from them
    const size_t nbody = ply.body.size();
    size_t need = 0;
    for (const Elem &e : ply.elems) {
        size_t rec = 0;
        for (const Prop &q : e.props)
            rec += ply.fmt == Fmt::Ascii ? 1 : (size_t)type_size(q.list() ? q.count_type : q.type);
        if (rec == 0) continue;
        MOF_REQUIRE((uint64_t)e.count <= nbody / rec, "PLY: element " + e.name + " count exceeds the file body");
        need += (size_t)e.count * rec;
        MOF_REQUIRE(need <= nbody, "PLY: element counts exceed the file body");
    }
    return ply;
}

struct Reader {
    const Ply &ply;
    size_t pos = 0;
    std::istringstream txt;
    explicit Reader(const Ply &p) : ply(p) {
        if (p.fmt == Fmt::Ascii) txt.str(std::string(p.body.begin(), p.body.end()));
    }
    // upper bound on the values still to be read (a list length must not exceed it)
    size_t remaining() {
        if (ply.fmt == Fmt::Ascii) {
            const std::streampos at = txt.tellg();
            return at < 0 ? 0 : ply.body.size() - (size_t)at;
        }
        return ply.body.size() - pos;
    }
    double scalar(const std::string &t) {
        if (ply.fmt == Fmt::Ascii) {
            double v;
            MOF_REQUIRE(static_cast<bool>(txt >> v), "PLY: truncated ascii body");
            return v;
        }
        const int sz = type_size(t);
        MOF_REQUIRE(pos + sz <= ply.body.size(), "PLY: truncated binary body");
        unsigned char b[8];
        std::memcpy(b, ply.body.data() + pos, sz);
        pos += sz;
        if (ply.fmt == Fmt::BinBE) std::reverse(b, b + sz);
        if (t == "char" || t == "int8") return (double)(int8_t)b[0];
        if (t == "uchar" || t == "uint8") return (double)b[0];
        if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return v; }
        if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return v; }
        if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return v; }
        if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return v; }
        if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
        double v;
        std::memcpy(&v, b, 8);
        return v;
    }
};

struct Surface {
    std::vector<float> points, normals;  // (N,3)
    std::vector<int64_t> tri;            // (M,3)
    int64_t N = 0, M = 0;
};

Surface read_ply(const char *path, bool want_data) {
    Ply ply = parse_header(path);
    Surface s;
    for (auto &e : ply.elems) {
        if (e.name == "vertex") s.N = e.count;
        if (e.name == "face") s.M = e.count;
    }
    MOF_REQUIRE(s.N > 0, "PLY: no vertices");
    bool has_n = false;
    for (auto &e : ply.elems)
        if (e.name == "vertex")
            for (auto &p : e.props) has_n |= (p.name == "nx");
    if (!want_data) {
        if (has_n) s.normals.resize(1);
        return s;
    }
    Reader rd(ply);
    s.points.assign(3 * s.N, 0.f);
    if (has_n) s.normals.assign(3 * s.N, 0.f);
    s.tri.reserve(3 * s.M);
    for (auto &e : ply.elems) {
        for (int64_t r = 0; r < e.count; ++r) {
            for (auto &p : e.props) {
                if (p.list()) {
                    const double nd = rd.scalar(p.count_type);
                    MOF_REQUIRE(nd >= 0.0 && nd <= (double)rd.remaining() && nd == std::floor(nd),
                                "PLY: bad list length");
                    const int64_t n = (int64_t)nd;
                    std::vector<double> ids(n);
                    for (int64_t k = 0; k < n; ++k) ids[k] = rd.scalar(p.type);
                    if (e.name == "face" && (p.name == "vertex_indices" || p.name == "vertex_index")) {
                        MOF_REQUIRE(n == 3, "PLY: only triangle faces are supported (S3 reshapes faces to (-1, 4))");
                        for (int64_t k = 0; k < 3; ++k) {
                            // range-checked as a double, before the integer cast
                            MOF_REQUIRE(ids[k] >= 0.0 && ids[k] < (double)s.N && ids[k] == std::floor(ids[k]),
                                        "PLY: face index out of range");
                            s.tri.push_back((int64_t)ids[k]);
                        }
                    }
                } else {
                    const double v = rd.scalar(p.type);
                    if (e.name != "vertex") continue;
                    int c = -1;
                    float *dst = nullptr;
                    if (p.name == "x" || p.name == "y" || p.name == "z") {
                        c = p.name[0] - 'x';
                        dst = s.points.data();
                    } else if (p.name == "nx" || p.name == "ny" || p.name == "nz") {
                        c = p.name[1] - 'x';
                        dst = s.normals.data();
                    }
                    if (dst) dst[3 * r + c] = (float)v;
                }
            }
        }
    }
    MOF_REQUIRE((int64_t)s.tri.size() == 3 * s.M, "PLY: face list incomplete");
    return s;
}

void tri_normal(const float *P, const int64_t *t, double n[3]) {
    double p0[3], p1[3], p2[3];
    for (int c = 0; c < 3; ++c) {
        p0[c] = P[3 * t[0] + c];
        p1[c] = P[3 * t[1] + c];
        p2[c] = P[3 * t[2] + c];
    }
    const double ax = p2[0] - p1[0], ay = p2[1] - p1[1], az = p2[2] - p1[2];
    const double bx = p0[0] - p1[0], by = p0[1] - p1[1], bz = p0[2] - p1[2];
    n[0] = ay * bz - az * by;
    n[1] = az * bx - ax * bz;
    n[2] = ax * by - ay * bx;
    const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (len != 0.0)
        for (int c = 0; c < 3; ++c) n[c] /= len;
}

}  // namespace
}  // namespace mof

int mof_ply_info(const char *path, int64_t *n_vertices, int64_t *n_faces, uint32_t *has_normals) {
    return mof_io_guard([&] {
        MOF_REQUIRE(path && n_vertices && n_faces, "NULL argument");
        mof::Surface s = mof::read_ply(path, false);
        *n_vertices = s.N;
        *n_faces = s.M;
        if (has_normals) *has_normals = s.normals.empty() ? 0u : 1u;
    });
}

int mof_ply_read(const char *path, float *points, int64_t *triangles, float *normals) {
    return mof_io_guard([&] {
        MOF_REQUIRE(path && points && triangles, "NULL argument");
        mof::Surface s = mof::read_ply(path, true);
        std::memcpy(points, s.points.data(), sizeof(float) * s.points.size());
        std::memcpy(triangles, s.tri.data(), sizeof(int64_t) * s.tri.size());
        if (normals && !s.normals.empty()) std::memcpy(normals, s.normals.data(), sizeof(float) * s.normals.size());
    });
}

int mof_point_normals(const float *points, const int64_t *triangles, int64_t N, int64_t M, float *normals) {
    return mof_io_guard([&] {
        MOF_REQUIRE(points && normals && (triangles || M == 0) && N >= 0 && M >= 0, "bad argument");
        std::vector<double> acc(3 * (size_t)N, 0.0);
        for (int64_t t = 0; t < M; ++t) {
            const int64_t *v = triangles + 3 * t;
            for (int k = 0; k < 3; ++k) MOF_REQUIRE(v[k] >= 0 && v[k] < N, "triangle index out of range");
            double n[3];
            mof::tri_normal(points, v, n);
            for (int k = 0; k < 3; ++k)
                for (int c = 0; c < 3; ++c) acc[3 * v[k] + c] += n[c];
        }
        for (int64_t i = 0; i < N; ++i) {
            double *n = &acc[3 * i];
            const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            if (len != 0.0)
                for (int c = 0; c < 3; ++c) n[c] /= len;
            for (int c = 0; c < 3; ++c) normals[3 * i + c] = (float)n[c];
        }
    });
}

int mof_cell_areas(const float *points, const int64_t *triangles, int64_t N, int64_t M, double *areas) {
    return mof_io_guard([&] {
        MOF_REQUIRE(points && areas && (triangles || M == 0) && N >= 0 && M >= 0, "bad argument");
        for (int64_t t = 0; t < M; ++t) {
            const int64_t *v = triangles + 3 * t;
            for (int k = 0; k < 3; ++k) MOF_REQUIRE(v[k] >= 0 && v[k] < N, "triangle index out of range");
            double a[3], b[3];
            for (int c = 0; c < 3; ++c) {
                a[c] = (double)points[3 * v[1] + c] - (double)points[3 * v[0] + c];
                b[c] = (double)points[3 * v[2] + c] - (double)points[3 * v[0] + c];
            }
            const double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
            areas[t] = 0.5 * std::sqrt(x * x + y * y + z * z);
        }
    });
}
