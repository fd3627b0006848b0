// loader.hip — host-side ASCII point parser for load_lidar_data's PCD / PLY data sections
// (utils/data_processing.py:43-104), the two formats the reference reads with per-line
// Python loops.  Host code only; no device work.
//
// Semantics reproduced for a data section starting at line `first` (0-based, the caller
// finds it with the reference's header rules): every line that is non-empty after
// stripping ASCII whitespace and has >= 3 whitespace-separated tokens contributes
// (float(tok0), float(tok1), float(tok2)); other lines are skipped.  max_lines < 0: to the
// end of the buffer (PCD); otherwise lines [first, first + max_lines) (PLY's vertex count).
// Python's float() is correctly rounded and so is glibc strtod on plain decimal / exponent
// / inf / nan tokens; a token strtod does not consume entirely (or one Python parses
// differently: '_' digit separators, hex, a leading '0x') makes the call return
// LIDAR_EPARSE so the caller falls back to the Python loop (and raises its exact error).
#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "common.hpp"

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// parse one token [p, e) -> *v; false when Python float() could disagree or fail
bool parse_token(const char *p, const char *e, double *v)
{
    const size_t len = (size_t)(e - p);
    if (len == 0 || len > 350) return false;
    char buf[352];
    for (size_t i = 0; i < len; ++i) {
        const char c = p[i];
        // Python-only / hex forms, and strtod's "nan(chars)", which Python's float() rejects: the
        // caller's Python loop then reproduces what the reference does with such a row
        if (c == '_' || c == 'x' || c == 'X' || c == 'p' || c == 'P' || c == '(') return false;
        buf[i] = c;
    }
    buf[len] = '\0';
    char *end = nullptr;
    errno = 0;
    const double d = strtod(buf, &end);
    if (end != buf + len) return false;
    *v = d;  // overflow to +-inf and underflow match Python float()
    return true;
}

// parse the lines of [p, end): 0 ok, LIDAR_EPARSE when a token needs Python's float()
int parse_lines(const char *p, const char *end, std::vector<double> &out)
{
    while (p < end) {
        const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        const char *le = nl ? nl : end;
        // bytes whose meaning differs between this scanner and Python's text mode / str.split()
        // (non-ASCII, \v \f \x1c-\x1f, a CR not ending the line): the Python path decides
        for (const char *c = p; c < le; ++c) {
            const unsigned char u = (unsigned char)*c;
            if (u >= 0x80 || u == 0x0b || u == 0x0c || (u >= 0x1c && u <= 0x1f) || (u == '\r' && c + 1 != le))
                return LIDAR_EPARSE;
        }
        const char *tb[3], *te[3];
        int nt = 0;
        const char *q = p;
        while (q < le && nt < 3) {
            while (q < le && is_space(*q)) ++q;
            if (q >= le) break;
            tb[nt] = q;
            while (q < le && !is_space(*q)) ++q;
            te[nt] = q;
            ++nt;
        }
        if (nt >= 3) {
            double v[3];
            for (int k = 0; k < 3; ++k)
                if (!parse_token(tb[k], te[k], &v[k])) return LIDAR_EPARSE;
            out.insert(out.end(), v, v + 3);
        }
        p = nl ? nl + 1 : end;
    }
    return 0;
}

}  // namespace

LIDAR_EXPORT int lidar_parse_ascii_xyz(const char *buf, int64_t len, int64_t first, int64_t max_lines,
                                       double *out, int64_t cap, int64_t *n_out)
{
    REQUIRE(buf && n_out && len >= 0 && first >= 0 && (cap == 0 || out), "lidar_parse_ascii_xyz: bad arguments");
    const char *p = buf, *end = buf + len;
    auto skip_lines = [&](const char *from, int64_t count) {
        for (int64_t l = 0; l < count && from < end; ++l) {
            const char *nl = static_cast<const char *>(memchr(from, '\n', (size_t)(end - from)));
            from = nl ? nl + 1 : end;
        }
        return from;
    };
    p = skip_lines(p, first);
    const char *stop = max_lines < 0 ? end : skip_lines(p, max_lines);
    // lines are independent: chunks cut at line ends, parsed in parallel, concatenated in order
    const int64_t bytes = stop - p;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nthr = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::min(hw, 16u), bytes / (1 << 20)}));
    std::vector<const char *> cut(nthr + 1);
    cut[0] = p;
    cut[nthr] = stop;
    for (int t = 1; t < nthr; ++t) {
        const char *c = p + bytes * t / nthr;
        if (c < cut[t - 1]) c = cut[t - 1];
        const char *nl = static_cast<const char *>(memchr(c, '\n', (size_t)(stop - c)));
        cut[t] = nl ? nl + 1 : stop;
    }
    std::vector<std::vector<double>> part(nthr);
    std::vector<int> rc(nthr, 0);
    std::vector<std::thread> th;
    for (int t = 1; t < nthr; ++t) th.emplace_back([&, t] { rc[t] = parse_lines(cut[t], cut[t + 1], part[t]); });
    rc[0] = parse_lines(cut[0], cut[1], part[0]);
    for (auto &x : th) x.join();
    int64_t n = 0;
    for (int t = 0; t < nthr; ++t) {
        if (rc[t]) return lidar::fail(LIDAR_EPARSE, "lidar_parse_ascii_xyz: token needs the Python parser");
        n += (int64_t)part[t].size() / 3;
    }
    if (n > cap) return lidar::fail(LIDAR_EINVAL, "lidar_parse_ascii_xyz: output capacity exceeded");
    double *o = out;
    for (int t = 0; t < nthr; ++t) {
        std::memcpy(o, part[t].data(), part[t].size() * sizeof(double));
        o += part[t].size();
    }
    *n_out = n;
    return LIDAR_OK;
}
