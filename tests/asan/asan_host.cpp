// asan_host.cpp -- AddressSanitizer driver for the host-only entry points of
// libmofhip (include/mof.h): the CSV writer/reader, the PLY reader, point
// normals / cell areas, the multigrid hierarchy probe, the RCB partition and
// the halo-plan diagnostic. Built by `make -C <csrc> asan` with the host
// halves of every source instrumented (no GPU is touched; device code is
// compiled but never launched). Well-formed inputs must round-trip; malformed
// ones must return an error status -- ASan aborts the run on any invalid
// access, and the test (tests/test_asan_host.py) requires exit status 0.
//
//     asan_host <scratch dir>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mof.h"

static int g_fail = 0;

#define CHECK(cond)                                                          \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                        \
        }                                                                    \
    } while (0)

static void write_file(const std::string &path, const std::string &text) {
    FILE *f = std::fopen(path.c_str(), "wb");
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
}

// closed torus mesh: n x m quads, two triangles each
static void torus(int n, int m, std::vector<double> &xyz, std::vector<int32_t> &tri) {
    xyz.clear();
    tri.clear();
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            const double u = 2 * M_PI * i / n, v = 2 * M_PI * j / m;
            xyz.push_back((3 + std::cos(v)) * std::cos(u));
            xyz.push_back((3 + std::cos(v)) * std::sin(u));
            xyz.push_back(std::sin(v));
        }
    auto id = [&](int i, int j) { return ((i + n) % n) * m + (j + m) % m; };
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            tri.insert(tri.end(), {id(i, j), id(i + 1, j), id(i + 1, j + 1)});
            tri.insert(tri.end(), {id(i, j), id(i + 1, j + 1), id(i, j + 1)});
        }
}

static void test_csv(const std::string &dir) {
    const int64_t R = 37, C = 11;
    std::vector<double> a(R * C);
    for (int64_t q = 0; q < R * C; ++q) a[q] = std::sin(0.37 * q) * std::pow(10.0, (q % 13) - 6);
    a[5] = NAN;
    a[6] = INFINITY;
    a[7] = -0.0;
    a[8] = 5e-324;
    a[9] = 1.7976931348623157e308;
    const std::string p = dir + "/ok.csv";
    CHECK(mof_csv_write(p.c_str(), a.data(), R, C, 3) == MOF_OK);
    int64_t r = 0, c = 0;
    CHECK(mof_csv_shape(p.c_str(), &r, &c) == MOF_OK && r == R && c == C);
    std::vector<double> b(R * C);
    CHECK(mof_csv_read(p.c_str(), b.data(), R, C, MOF_CSV_ROUND_TRIP, 4) == MOF_OK);
    for (int64_t q = 0; q < R * C; ++q) CHECK((std::isnan(a[q]) && std::isnan(b[q])) || a[q] == b[q]);
    CHECK(mof_csv_read(p.c_str(), b.data(), R, C, 0, 1) == MOF_OK);
    // wrong shape, missing file, empty file, ragged and garbage rows
    CHECK(mof_csv_read(p.c_str(), b.data(), R + 1, C, 0, 2) != MOF_OK);
    CHECK(mof_csv_shape((dir + "/missing.csv").c_str(), &r, &c) != MOF_OK);
    const std::string e = dir + "/empty.csv";
    write_file(e, "");
    CHECK(mof_csv_shape(e.c_str(), &r, &c) == MOF_OK && r == 0);
    CHECK(mof_csv_read(e.c_str(), nullptr, 0, 0, 0, 2) == MOF_OK);
    write_file(e, ",0,1\n");
    CHECK(mof_csv_shape(e.c_str(), &r, &c) == MOF_OK && r == 0);
    const std::string g = dir + "/bad.csv";
    const char *bad[] = {
        ",0,1,2\n0,1.5,2.5\n",               // short row
        ",0,1,2\n0,1,2,x3\n",                 // garbage token
        ",0,1,2\n0,1e,2,3\n",                 // dangling exponent
        ",0,1,2\n0,1,2,3e99999999999999999\n", // absurd exponent
        ",0,1,2\n0,--1,2,3\n",
        ",0,1,2\n0,1,2,3",                    // no final newline (valid)
        ",0,1,2\r\n0,1,2,3\r\n",              // CRLF (valid)
        ",0,1,2\n0,.,2,3\n",
        ",0,1,2\n\n\n0,1,2,3\n\n",           // blank lines (valid)
    };
    for (const char *t : bad) {
        write_file(g, t);
        if (mof_csv_shape(g.c_str(), &r, &c) != MOF_OK) continue;
        std::vector<double> o((size_t)std::max<int64_t>(1, r * c));
        (void)mof_csv_read(g.c_str(), o.data(), r, c, 0, 2);
        (void)mof_csv_read(g.c_str(), o.data(), r, c, MOF_CSV_ROUND_TRIP, 1);
    }
    // a long row of many threads' chunks
    std::string big = ",0\n";
    for (int q = 0; q < 200000; ++q) big += std::to_string(q) + "," + std::to_string(q * 0.5) + "\n";
    write_file(g, big);
    CHECK(mof_csv_shape(g.c_str(), &r, &c) == MOF_OK && r == 200000 && c == 1);
    std::vector<double> o(r);
    CHECK(mof_csv_read(g.c_str(), o.data(), r, c, 0, 8) == MOF_OK && o[12345] == 6172.5);
}

static void test_ply(const std::string &dir) {
    const std::string p = dir + "/t.ply";
    const std::string hdr =
        "ply\nformat ascii 1.0\nelement vertex 4\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 4\nproperty list uchar int vertex_indices\nend_header\n";
    write_file(p, hdr + "0 0 0\n1 0 0\n0 1 0\n0 0 1\n3 0 2 1\n3 0 1 3\n3 0 3 2\n3 1 2 3\n");
    int64_t n = 0, m = 0;
    uint32_t hn = 0;
    CHECK(mof_ply_info(p.c_str(), &n, &m, &hn) == MOF_OK && n == 4 && m == 4 && hn == 0);
    std::vector<float> pts(12), nrm(12);
    std::vector<int64_t> tri(12);
    CHECK(mof_ply_read(p.c_str(), pts.data(), tri.data(), nullptr) == MOF_OK && tri[11] == 3);
    CHECK(mof_point_normals(pts.data(), tri.data(), 4, 4, nrm.data()) == MOF_OK);
    std::vector<double> area(4);
    CHECK(mof_cell_areas(pts.data(), tri.data(), 4, 4, area.data()) == MOF_OK && std::fabs(area[0] - 0.5) < 1e-7);
    tri[5] = 9;  // out of range
    CHECK(mof_point_normals(pts.data(), tri.data(), 4, 4, nrm.data()) != MOF_OK);
    CHECK(mof_cell_areas(pts.data(), tri.data(), 4, 4, area.data()) != MOF_OK);
    // binary little endian with normals
    {
        std::string b =
            "ply\nformat binary_little_endian 1.0\nelement vertex 3\nproperty float x\nproperty float y\n"
            "property float z\nproperty float nx\nproperty float ny\nproperty float nz\nelement face 1\n"
            "property list uchar int vertex_indices\nend_header\n";
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 6; ++k) {
                const float f = (float)(v == k) + 0.25f * k;
                b.append(reinterpret_cast<const char *>(&f), 4);
            }
        b.push_back((char)3);
        for (int32_t v : {0, 1, 2}) b.append(reinterpret_cast<const char *>(&v), 4);
        write_file(p, b);
        CHECK(mof_ply_info(p.c_str(), &n, &m, &hn) == MOF_OK && n == 3 && m == 1 && hn == 1);
        CHECK(mof_ply_read(p.c_str(), pts.data(), tri.data(), nrm.data()) == MOF_OK && tri[2] == 2);
        write_file(p, b.substr(0, b.size() - 3));  // truncated body
        CHECK(mof_ply_read(p.c_str(), pts.data(), tri.data(), nrm.data()) != MOF_OK);
    }
    const char *bad[] = {
        "",
        "plyx\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\n",  // no end_header
        "ply\nformat ascii 1.0\nproperty float x\nend_header\n",
        "ply\nformat weird 1.0\nend_header\n",
        "ply\nformat ascii 1.0\nelement vertex 1000000000000\nproperty float x\nend_header\n0\n",
        "ply\nformat binary_little_endian 1.0\nelement vertex 2000000000\nproperty double x\nend_header\nabc",
        "ply\nformat ascii 1.0\nelement vertex -5\nproperty float x\nend_header\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face -2\nproperty list uchar int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 1\nproperty list uchar int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n4 0 1 2 0\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 1\nproperty list uchar int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n3 0 1 7\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 1\nproperty list int int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n-7 0 1 2\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 1\nproperty list int int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n1e300 0 1 2\n",
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
        "element face 1\nproperty list uchar int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n3 0 1 nan\n",
        "ply\nformat ascii 1.0\nelement vertex 2\nproperty float x\nelement vertex 9\nproperty float x\n"
        "end_header\n0 1 2 3 4 5 6 7 8 9 10\n",  // two vertex elements
        "ply\nformat ascii 1.0\nelement vertex 3\nproperty mystery x\nend_header\n1 2 3\n",
    };
    for (const char *t : bad) {
        write_file(p, t);
        if (mof_ply_info(p.c_str(), &n, &m, &hn) != MOF_OK) continue;
        if (n <= 0 || n > 1000 || m < 0 || m > 1000) continue;  // the reader itself must reject these
        std::vector<float> P(3 * n + 3), Nn(3 * n + 3);
        std::vector<int64_t> Tt(3 * m + 3);
        (void)mof_ply_read(p.c_str(), P.data(), Tt.data(), Nn.data());
    }
    // counts beyond the body must be rejected before any allocation
    for (const char *t : {bad[5], bad[6], bad[7], bad[8], bad[14]}) {
        write_file(p, t);
        std::vector<float> P(64), Nn(64);
        std::vector<int64_t> Tt(64);
        CHECK(mof_ply_info(p.c_str(), &n, &m, &hn) != MOF_OK ||
              mof_ply_read(p.c_str(), P.data(), Tt.data(), Nn.data()) != MOF_OK);
    }
}

static void test_mesh_host(void) {
    std::vector<double> xyz;
    std::vector<int32_t> tri;
    torus(40, 24, xyz, tri);
    const int32_t N = (int32_t)(xyz.size() / 3), M = (int32_t)(tri.size() / 3);
    // any orthonormal tangent basis works for the probe
    std::vector<double> e(6 * (size_t)N);
    for (int32_t i = 0; i < N; ++i) {
        const double x = xyz[3 * i], y = xyz[3 * i + 1], r = std::hypot(x, y);
        const double t0[3] = {-y / r, x / r, 0.0};
        e[6 * i + 0] = t0[0];
        e[6 * i + 1] = t0[1];
        e[6 * i + 2] = t0[2];
        e[6 * i + 3] = 0.0;
        e[6 * i + 4] = 0.0;
        e[6 * i + 5] = 1.0;
    }
    int32_t nl = 0, ln[16];
    double qerr = 1.0;
    CHECK(mof_amg_probe(tri.data(), e.data(), N, M, &nl, ln, &qerr, nullptr) == MOF_OK && nl >= 2 && ln[0] == N);
    CHECK(qerr < 1e-5);
    std::vector<int32_t> badtri = tri;
    badtri[7] = N + 3;
    CHECK(mof_amg_probe(badtri.data(), e.data(), N, M, &nl, ln, &qerr, nullptr) != MOF_OK);
    for (int32_t P : {1, 2, 3, 8}) {
        std::vector<int32_t> part(N, -1);
        CHECK(mof_partition_rcb(xyz.data(), N, P, part.data()) == MOF_OK);
        std::vector<int32_t> cnt(P, 0);
        for (int32_t v : part) {
            CHECK(v >= 0 && v < P);
            if (v >= 0 && v < P) cnt[v]++;
        }
        for (int32_t k = 0; k < P; ++k) CHECK(cnt[k] == N / P || cnt[k] == (N + P - 1) / P);
        std::vector<int32_t> own(P), ghost(P), nbr(P), ntri(P);
        std::vector<int64_t> snd(P);
        CHECK(mof_dd_plan_info(tri.data(), N, M, P, part.data(), own.data(), ghost.data(), nbr.data(), ntri.data(),
                               snd.data()) == MOF_OK);
        int64_t tot = 0;
        for (int32_t k = 0; k < P; ++k) tot += own[k];
        CHECK(tot == N);
        part[0] = P;  // out-of-range part id
        CHECK(mof_dd_plan_info(tri.data(), N, M, P, part.data(), own.data(), ghost.data(), nbr.data(), ntri.data(),
                               snd.data()) != MOF_OK);
    }
    CHECK(mof_partition_rcb(xyz.data(), N, 0, nullptr) != MOF_OK);
    CHECK(mof_xcd_map_check(160, 256, 8) == MOF_OK && mof_xcd_map_check(3, 5, 32) == MOF_OK);
}

int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    test_csv(dir);
    test_ply(dir);
    test_mesh_host();
    std::printf("asan_host: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
