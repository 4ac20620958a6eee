// mof_io.cpp -- SURVEY.md §8(f)2: the S3 CSV files, natively and in parallel.
//
// The reference writes e (N,6) and V_k (T-1, 2N) with
//   pd.DataFrame(data.reshape(rows, -1)).to_csv(path)
// (compute_optical_flow.py:314-320) and reads the potentials with
//   pd.read_csv(path, sep=',', header='infer', index_col=0).values
// (compute_optical_flow.py:203-207). At 160k vertices x 5000 timesteps the
// V_k file is ~13 GB of text, written by one Python thread.
//
// mof_csv_write produces the same bytes as pandas 2.x to_csv: a header line
// ",0,1,...,cols-1", then "row,v0,v1,..." per row, every float in Python's
// repr (shortest round-trip digits; fixed notation when the decimal exponent
// is in [-4, 16), else d.ddde+XX), NaN as an empty field, +-inf as "inf" /
// "-inf", "\n" line ends. Rows are formatted by a pool of host threads in
// bounded blocks and written in order.
//
// mof_csv_shape / mof_csv_read parse such a file (header line skipped, the
// first field of each row dropped as the index), chunked over threads on a
// memory-mapped file, with pandas' default float parser restated bit for bit
// (or correctly rounded std::from_chars with MOF_CSV_ROUND_TRIP, =
// float_precision='round_trip'); empty fields and pandas' NA strings read as
// NaN.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "mof_internal.h"

namespace mof {
namespace {

// threads > 0: as given; else MOF_IO_THREADS, else OMP_NUM_THREADS (the
// process's CPU share on shared hosts), else all cores; at most 64.
int32_t pool_size(int32_t threads) {
    if (threads > 0) return std::min(threads, 256);
    if (const int32_t t = knob_threads(64)) return t;
    const unsigned hc = std::thread::hardware_concurrency();
    return (int32_t)std::min(64u, std::max(1u, hc));
}

template <typename F>
void parallel_for(int32_t nthreads, int64_t n, F &&body) {
    if (n <= 0) return;
    const int32_t T = (int32_t)std::min<int64_t>(nthreads, n);
    if (T <= 1) {
        body(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(T);
    for (int32_t t = 0; t < T; ++t) {
        const int64_t a = n * t / T, b = n * (t + 1) / T;
        pool.emplace_back([&body, t, a, b] { body(t, a, b); });
    }
    for (auto &th : pool) th.join();
}

// Python repr of a finite or infinite double (NaN handled by the caller).
// Returns the number of chars written to out (needs <= 32 bytes).
int py_repr(double x, char *out) {
    char *o = out;
    if (std::isinf(x)) {
        if (x < 0) *o++ = '-';
        std::memcpy(o, "inf", 3);
        return (int)(o + 3 - out);
    }
    char buf[40];
    // shortest round-trip digits, scientific: [-]d[.ddd]e[+-]XX
    const auto res = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
    const char *p = buf, *end = res.ptr;
    if (*p == '-') {
        *o++ = '-';
        ++p;
    }
    char dig[20];
    int nd = 0;
    for (; p < end && *p != 'e'; ++p)
        if (*p != '.') dig[nd++] = *p;
    int ex = 0;
    std::from_chars(p + 1 + (p[1] == '+'), end, ex);
    const int decpt = ex + 1;  // value = 0.d1d2... x 10^decpt
    if (decpt <= -4 || decpt > 16) {
        *o++ = dig[0];
        if (nd > 1) {
            *o++ = '.';
            std::memcpy(o, dig + 1, nd - 1);
            o += nd - 1;
        }
        *o++ = 'e';
        *o++ = ex < 0 ? '-' : '+';
        const int ae = ex < 0 ? -ex : ex;
        if (ae < 10) *o++ = '0';
        o = std::to_chars(o, o + 4, ae).ptr;
    } else if (decpt <= 0) {
        *o++ = '0';
        *o++ = '.';
        for (int k = 0; k < -decpt; ++k) *o++ = '0';
        std::memcpy(o, dig, nd);
        o += nd;
    } else if (decpt >= nd) {
        std::memcpy(o, dig, nd);
        o += nd;
        for (int k = nd; k < decpt; ++k) *o++ = '0';
        *o++ = '.';
        *o++ = '0';
    } else {
        std::memcpy(o, dig, decpt);
        o += decpt;
        *o++ = '.';
        std::memcpy(o, dig + decpt, nd - decpt);
        o += nd - decpt;
    }
    return (int)(o - out);
}

void format_rows(const double *data, int64_t cols, int64_t r0, int64_t r1, std::string &s) {
    s.clear();
    s.reserve((size_t)((r1 - r0) * (cols * 24 + 12)));
    char tmp[48];
    for (int64_t r = r0; r < r1; ++r) {
        s.append(tmp, std::to_chars(tmp, tmp + sizeof tmp, r).ptr);
        const double *row = data + r * cols;
        for (int64_t c = 0; c < cols; ++c) {
            s.push_back(',');
            const double v = row[c];
            if (!std::isnan(v)) s.append(tmp, (size_t)py_repr(v, tmp));
        }
        s.push_back('\n');
    }
}

void write_all(int fd, const char *p, size_t n) {
    while (n > 0) {
        const ssize_t w = ::write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            throw Error{MOF_E_ARG, std::string("write failed: ") + std::strerror(errno)};
        }
        p += w;
        n -= (size_t)w;
    }
}

struct Mapped {
    const char *p = nullptr;
    size_t n = 0;
    int fd = -1;
    explicit Mapped(const char *path) {
        fd = ::open(path, O_RDONLY);
        MOF_REQUIRE(fd >= 0, std::string("cannot open ") + path + ": " + std::strerror(errno));
        struct stat st;
        MOF_REQUIRE(::fstat(fd, &st) == 0, "fstat failed");
        n = (size_t)st.st_size;
        if (n > 0) {
            void *m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            MOF_REQUIRE(m != MAP_FAILED, std::string("mmap failed: ") + std::strerror(errno));
            p = static_cast<const char *>(m);
            ::madvise(m, n, MADV_SEQUENTIAL);
        }
    }
    ~Mapped() {
        if (p) ::munmap(const_cast<char *>(p), n);
        if (fd >= 0) ::close(fd);
    }
};

// [begin, end) of the data lines (after the header line)
void data_region(const Mapped &f, const char *&b, const char *&e) {
    if (f.n == 0) {  // empty file: nothing mapped
        b = e = nullptr;
        return;
    }
    const char *nl = static_cast<const char *>(std::memchr(f.p, '\n', f.n));
    b = nl ? nl + 1 : f.p + f.n;
    e = f.p + f.n;
}

int64_t count_fields(const char *b, const char *e) {
    int64_t n = 1;
    for (const char *p = b; p < e && *p != '\n' && *p != '\r'; ++p) n += (*p == ',');
    return n;
}

// start of the first line at or after p
const char *line_start(const char *b, const char *e, const char *p) {
    if (p <= b) return b;
    const char *nl = static_cast<const char *>(std::memchr(p - 1, '\n', (size_t)(e - (p - 1))));
    return nl ? nl + 1 : e;
}

bool blank_tail(const char *p, const char *e) {
    for (; p < e; ++p)
        if (*p != '\n' && *p != '\r' && *p != ' ') return false;
    return true;
}


// pandas' default float parser (read_csv float_precision=None/'high':
// precise_xstrtod in pandas/_libs/src/parser/tokenizer.c, pandas 2.x),
// restated so mof_csv_read returns the reference's values bit for bit: at
// most 17 significant characters are accumulated as `number * 10 + digit`
// in double (leading zeros count), later integer digits raise the exponent,
// later decimals are dropped, then one multiply / divide by an exact power
// of ten (two divides for subnormal exponents). Not correctly rounded.
const double kPow10[309] = {
    1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16,
    1e17, 1e18, 1e19, 1e20, 1e21, 1e22, 1e23, 1e24, 1e25, 1e26, 1e27, 1e28, 1e29, 1e30, 1e31, 1e32,
    1e33, 1e34, 1e35, 1e36, 1e37, 1e38, 1e39, 1e40, 1e41, 1e42, 1e43, 1e44, 1e45, 1e46, 1e47, 1e48,
    1e49, 1e50, 1e51, 1e52, 1e53, 1e54, 1e55, 1e56, 1e57, 1e58, 1e59, 1e60, 1e61, 1e62, 1e63, 1e64,
    1e65, 1e66, 1e67, 1e68, 1e69, 1e70, 1e71, 1e72, 1e73, 1e74, 1e75, 1e76, 1e77, 1e78, 1e79, 1e80,
    1e81, 1e82, 1e83, 1e84, 1e85, 1e86, 1e87, 1e88, 1e89, 1e90, 1e91, 1e92, 1e93, 1e94, 1e95, 1e96,
    1e97, 1e98, 1e99, 1e100, 1e101, 1e102, 1e103, 1e104, 1e105, 1e106, 1e107, 1e108, 1e109, 1e110,
    1e111, 1e112, 1e113, 1e114, 1e115, 1e116, 1e117, 1e118, 1e119, 1e120, 1e121, 1e122, 1e123,
    1e124, 1e125, 1e126, 1e127, 1e128, 1e129, 1e130, 1e131, 1e132, 1e133, 1e134, 1e135, 1e136,
    1e137, 1e138, 1e139, 1e140, 1e141, 1e142, 1e143, 1e144, 1e145, 1e146, 1e147, 1e148, 1e149,
    1e150, 1e151, 1e152, 1e153, 1e154, 1e155, 1e156, 1e157, 1e158, 1e159, 1e160, 1e161, 1e162,
    1e163, 1e164, 1e165, 1e166, 1e167, 1e168, 1e169, 1e170, 1e171, 1e172, 1e173, 1e174, 1e175,
    1e176, 1e177, 1e178, 1e179, 1e180, 1e181, 1e182, 1e183, 1e184, 1e185, 1e186, 1e187, 1e188,
    1e189, 1e190, 1e191, 1e192, 1e193, 1e194, 1e195, 1e196, 1e197, 1e198, 1e199, 1e200, 1e201,
    1e202, 1e203, 1e204, 1e205, 1e206, 1e207, 1e208, 1e209, 1e210, 1e211, 1e212, 1e213, 1e214,
    1e215, 1e216, 1e217, 1e218, 1e219, 1e220, 1e221, 1e222, 1e223, 1e224, 1e225, 1e226, 1e227,
    1e228, 1e229, 1e230, 1e231, 1e232, 1e233, 1e234, 1e235, 1e236, 1e237, 1e238, 1e239, 1e240,
    1e241, 1e242, 1e243, 1e244, 1e245, 1e246, 1e247, 1e248, 1e249, 1e250, 1e251, 1e252, 1e253,
    1e254, 1e255, 1e256, 1e257, 1e258, 1e259, 1e260, 1e261, 1e262, 1e263, 1e264, 1e265, 1e266,
    1e267, 1e268, 1e269, 1e270, 1e271, 1e272, 1e273, 1e274, 1e275, 1e276, 1e277, 1e278, 1e279,
    1e280, 1e281, 1e282, 1e283, 1e284, 1e285, 1e286, 1e287, 1e288, 1e289, 1e290, 1e291, 1e292,
    1e293, 1e294, 1e295, 1e296, 1e297, 1e298, 1e299, 1e300, 1e301, 1e302, 1e303, 1e304, 1e305,
    1e306, 1e307, 1e308};

bool pandas_high_strtod(const char *p, const char *end, double &out) {
    bool neg = false;
    if (p < end && (*p == '-' || *p == '+')) neg = (*p++ == '-');
    double number = 0.0;
    int exponent = 0, nd = 0, ndec = 0;
    constexpr int kMaxDigits = 17;
    while (p < end && *p >= '0' && *p <= '9') {
        if (nd < kMaxDigits) {
            number = number * 10. + (*p - '0');
            ++nd;
        } else {
            ++exponent;
        }
        ++p;
    }
    if (p < end && *p == '.') {
        ++p;
        while (nd < kMaxDigits && p < end && *p >= '0' && *p <= '9') {
            number = number * 10. + (*p - '0');
            ++p;
            ++nd;
            ++ndec;
        }
        while (p < end && *p >= '0' && *p <= '9') ++p;
        exponent -= ndec;
    }
    if (nd == 0) return false;
    if (neg) number = -number;
    if (p < end && (*p == 'e' || *p == 'E')) {
        const char *q = p + 1;
        bool eneg = false;
        if (q < end && (*q == '-' || *q == '+')) eneg = (*q++ == '-');
        int n = 0, ed = 0;
        while (ed < kMaxDigits && q < end && *q >= '0' && *q <= '9') {
            // saturate: any |exponent| past 616 gives inf / 0 either way, and
            // 17 digits would overflow an int
            n = n < 100000000 ? n * 10 + (*q - '0') : n;
            ++ed;
            ++q;
        }
        if (ed > 0) {
            exponent += eneg ? -n : n;
            p = q;
        }
    }
    if (p != end) return false;
    if (exponent > 308) {
        number = number < 0 ? -HUGE_VAL : HUGE_VAL;
    } else if (exponent > 0) {
        number *= kPow10[exponent];
    } else if (exponent < -308) {
        if (exponent < -616) {
            number = 0.;
        } else {
            number /= kPow10[-308 - exponent];
            number /= kPow10[308];
        }
    } else {
        number /= kPow10[-exponent];
    }
    out = number;
    return true;
}

// pandas' default NA strings and the infinities its converter accepts
bool special_value(const char *s0, const char *s1, double &out) {
    const std::string v(s0, s1);
    static const char *na[] = {"NaN", "nan", "NA", "N/A", "n/a", "NULL", "null", "#N/A", "#NA", "-nan",
                               "-NaN", "1.#IND", "-1.#IND", "1.#QNAN", "-1.#QNAN", "<NA>", "None",
                               "#N/A N/A"};
    for (const char *x : na)
        if (v == x) {
            out = std::numeric_limits<double>::quiet_NaN();
            return true;
        }
    std::string l;
    for (char c : v) l.push_back((char)std::tolower((unsigned char)c));
    if (l == "inf" || l == "+inf" || l == "infinity" || l == "+infinity") {
        out = HUGE_VAL;
        return true;
    }
    if (l == "-inf" || l == "-infinity") {
        out = -HUGE_VAL;
        return true;
    }
    return false;
}

}  // namespace
}  // namespace mof

int mof_io_guard(const std::function<void()> &f);  // mof_abi.cpp: status + mof_last_error

int mof_csv_write(const char *path, const double *data, int64_t rows, int64_t cols, int32_t threads) {
    return mof_io_guard([&] {
        MOF_REQUIRE(path && (data || rows * cols == 0) && rows >= 0 && cols >= 0, "bad argument");
        const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        MOF_REQUIRE(fd >= 0, std::string("cannot create ") + path + ": " + std::strerror(errno));
        try {
            std::string head;
            char tmp[32];
            for (int64_t c = 0; c < cols; ++c) {
                head.push_back(',');
                head.append(tmp, std::to_chars(tmp, tmp + sizeof tmp, c).ptr);
            }
            head.push_back('\n');
            mof::write_all(fd, head.data(), head.size());
            const int32_t T = mof::pool_size(threads);
            // blocks of ~32 MB of text per thread, written in row order
            const int64_t per = std::max<int64_t>(1, (int64_t)(32 << 20) / std::max<int64_t>(1, cols * 22));
            std::vector<std::string> bufs(T);
            for (int64_t r0 = 0; r0 < rows; r0 += per * T) {
                const int64_t r1 = std::min(rows, r0 + per * T);
                mof::parallel_for(T, r1 - r0, [&](int32_t t, int64_t a, int64_t b) {
                    mof::format_rows(data, cols, r0 + a, r0 + b, bufs[t]);
                });
                const int32_t used = (int32_t)std::min<int64_t>(T, r1 - r0);
                for (int32_t t = 0; t < used; ++t) mof::write_all(fd, bufs[t].data(), bufs[t].size());
            }
        } catch (...) {
            ::close(fd);
            throw;
        }
        MOF_REQUIRE(::close(fd) == 0, std::string("close failed: ") + std::strerror(errno));
    });
}

int mof_csv_shape(const char *path, int64_t *rows, int64_t *cols) {
    return mof_io_guard([&] {
        MOF_REQUIRE(path && rows && cols, "NULL argument");
        mof::Mapped f(path);
        const char *b, *e;
        mof::data_region(f, b, e);
        int64_t n = 0;
        for (const char *p = b; p < e;) {
            const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(e - p)));
            const char *le = nl ? nl : e;
            if (!mof::blank_tail(p, le)) ++n;
            p = nl ? nl + 1 : e;
        }
        *rows = n;
        *cols = n > 0 ? mof::count_fields(b, e) - 1 : 0;
    });
}

int mof_csv_read(const char *path, double *out, int64_t rows, int64_t cols, uint32_t flags,
                 int32_t threads) {
    const bool round_trip = (flags & MOF_CSV_ROUND_TRIP) != 0;
    return mof_io_guard([&] {
        MOF_REQUIRE(path && (out || rows * cols == 0) && rows >= 0 && cols >= 0, "bad argument");
        mof::Mapped f(path);
        const char *b, *e;
        mof::data_region(f, b, e);
        const int32_t T = mof::pool_size(threads);
        // chunk boundaries at line starts; each chunk counts its rows first
        const int32_t C = (int32_t)std::max<int64_t>(1, std::min<int64_t>(4 * T, (e - b) / (1 << 16) + 1));
        std::vector<const char *> cut(C + 1);
        for (int32_t k = 0; k <= C; ++k) cut[k] = mof::line_start(b, e, b + (e - b) * k / C);
        std::vector<int64_t> nrow(C + 1, 0);
        mof::parallel_for(T, C, [&](int32_t, int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; ++k) {
                int64_t n = 0;
                for (const char *p = cut[k]; p < cut[k + 1];) {
                    const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(cut[k + 1] - p)));
                    const char *le = nl ? nl : cut[k + 1];
                    if (!mof::blank_tail(p, le)) ++n;
                    p = nl ? nl + 1 : cut[k + 1];
                }
                nrow[k + 1] = n;
            }
        });
        for (int32_t k = 0; k < C; ++k) nrow[k + 1] += nrow[k];
        MOF_REQUIRE(nrow[C] == rows, "row count mismatch (call mof_csv_shape first)");
        std::vector<std::string> err(C);
        mof::parallel_for(T, C, [&](int32_t, int64_t k0, int64_t k1) {
            const double nan = std::numeric_limits<double>::quiet_NaN();
            for (int64_t k = k0; k < k1; ++k) {
                int64_t r = nrow[k];
                for (const char *p = cut[k]; p < cut[k + 1] && err[k].empty();) {
                    const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(cut[k + 1] - p)));
                    const char *le = nl ? nl : cut[k + 1];
                    const char *next = nl ? nl + 1 : cut[k + 1];
                    if (le > p && le[-1] == '\r') --le;
                    if (mof::blank_tail(p, le)) {
                        p = next;
                        continue;
                    }
                    const char *q = static_cast<const char *>(std::memchr(p, ',', (size_t)(le - p)));
                    q = q ? q + 1 : le;  // skip the index field
                    double *o = out + r * cols;
                    int64_t c = 0;
                    while (c < cols) {
                        const char *fe = static_cast<const char *>(std::memchr(q, ',', (size_t)(le - q)));
                        if (!fe) fe = le;
                        const char *s0 = q, *s1 = fe;
                        while (s0 < s1 && *s0 == ' ') ++s0;
                        while (s1 > s0 && s1[-1] == ' ') --s1;
                        bool ok = true;
                        if (s0 == s1) {
                            o[c] = nan;
                        } else if (round_trip) {
                            const char *t0 = s0 + (*s0 == '+');
                            const auto res = std::from_chars(t0, s1, o[c]);
                            ok = (res.ec == std::errc() && res.ptr == s1) || mof::special_value(s0, s1, o[c]);
                        } else {
                            ok = mof::pandas_high_strtod(s0, s1, o[c]) || mof::special_value(s0, s1, o[c]);
                        }
                        if (!ok) {
                            err[k] = "cannot parse field " + std::to_string(c + 1) + " of data row " +
                                     std::to_string(r);
                            break;
                        }
                        ++c;
                        if (fe == le) break;
                        q = fe + 1;
                    }
                    if (err[k].empty() && c != cols)
                        err[k] = "data row " + std::to_string(r) + " has " + std::to_string(c) +
                                 " values, expected " + std::to_string(cols);
                    ++r;
                    p = next;
                }
            }
        });
        for (auto &m : err) MOF_REQUIRE(m.empty(), m);
    });
}
