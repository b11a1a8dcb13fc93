// obj_parse.cpp -- load_model_data (OBJ_loader.cpp:278-360) with the reference's number parser
// (utilities/parser.h:38-205), single- or multi-threaded.
//
// The reference splits the file into `threads` newline-aligned chunks (OBJ_loader.cpp:298-331),
// parses them on its thread pool (parse_chunks, :32-176), joins the per-chunk arrays in chunk
// order (join_chunks, :190-227) and only then resolves relative indices (prep_model_data,
// :229-267). A line never spans two chunks and its parse never reads past its '\n', so the
// joined arrays are the single-pass arrays: the threaded load is bit-identical to threads = 1.
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "host_scene.h"

using namespace atr;

namespace {

// A cursor over OBJ text in which every line ends in '\n'. A NUL byte reads as a blank (the
// reference's C-string scan would stop at it; blanks keep the rest of the line parseable).
struct Cursor {
    const char* p;
    bool at(char c) const { return *p == c || (c == ' ' && *p == '\0'); }
    void skip_blanks() { while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\0') ++p; }  // parser.h:4-35
    void to_next_line() { while (*p != '\n') ++p; ++p; }
    static bool digit(char c) { return c >= '0' && c <= '9'; }

    // parse_int (parser.h:38-65); int32 overflow wraps (the reference's is UB)
    int32_t integer() {
        skip_blanks();
        uint32_t sgn = 1u;
        if (*p == '+') ++p;
        else if (*p == '-') { sgn = 0xFFFFFFFFu; ++p; }
        uint32_t v = 0;
        while (digit(*p)) v = v * 10u + uint32_t(*p++ - '0');
        return int32_t(v * sgn);
    }

    // parse_f64 (parser.h:113-191): integer mantissa of all digits, one f64 multiply by the
    // power-of-ten table entry for (exponent - fraction digits), table range 1e-28..1e19.
    double real() {
        static const double kPow10[48] = {
            1.0e-28, 1.0e-27, 1.0e-26, 1.0e-25, 1.0e-24, 1.0e-23, 1.0e-22, 1.0e-21, 1.0e-20, 1.0e-19,
            1.0e-18, 1.0e-17, 1.0e-16, 1.0e-15, 1.0e-14, 1.0e-13, 1.0e-12, 1.0e-11, 1.0e-10, 1.0e-9,
            1.0e-8,  1.0e-7,  1.0e-6,  1.0e-5,  1.0e-4,  1.0e-3,  1.0e-2,  1.0e-1,  1.0e0,   1.0e1,
            1.0e2,   1.0e3,   1.0e4,   1.0e5,   1.0e6,   1.0e7,   1.0e8,   1.0e9,   1.0e10,  1.0e11,
            1.0e12,  1.0e13,  1.0e14,  1.0e15,  1.0e16,  1.0e17,  1.0e18,  1.0e19};
        skip_blanks();
        double sgn = 1.0;
        if (*p == '+') ++p;
        else if (*p == '-') { sgn = -1.0; ++p; }
        uint64_t mant = 0;
        while (digit(*p)) mant = mant * 10u + uint64_t(*p++ - '0');
        if (*p == '.') ++p;
        uint64_t frac = 0;
        int ndig = 0;
        while (digit(*p)) { frac = frac * 10u + uint64_t(*p++ - '0'); ++ndig; }
        uint64_t scale10 = 1;
        for (int i = 0; i < (ndig > 19 ? 19 : ndig); ++i) scale10 *= 10u;
        mant = mant * scale10 + frac;
        int e = 0;
        if (*p == 'e' || *p == 'E') {
            ++p;
            int es = 1;
            if (*p == '+') ++p;
            else if (*p == '-') { es = -1; ++p; }
            while (digit(*p)) e = 10 * e + (*p++ - '0');
            e *= es;
        }
        e -= ndig;
        double v = double(mant) * sgn;
        if (e < -28 || e > 19) e = 0;
        return v * kPow10[e + 28];
    }
    V3 vec3() {  // parse_vec3f (parser.h:194-205)
        float x = float(real());
        float y = float(real());
        float z = float(real());
        return mk(x, y, z);
    }
};

// parse_chunks (OBJ_loader.cpp:32-176) over whole lines [p, end): raw 1-based / relative indices.
void parse_lines(const char* p, const char* end, HostMesh& m) {
    {   // size the arrays first (one pass over the line starts): no regrowth while parsing
        size_t nv = 0, nt = 0, nn = 0, nf = 0;
        for (const char* q = p; q < end;) {
            if (q[0] == 'v') {
                if (q[1] == ' ') ++nv;
                else if (q[1] == 't') ++nt;
                else if (q[1] == 'n') ++nn;
            } else if (q[0] == 'f') {
                ++nf;
            }
            const void* nl = std::memchr(q, '\n', size_t(end - q));
            q = nl ? static_cast<const char*>(nl) + 1 : end;
        }
        m.vertices.reserve(nv); m.texcoords.reserve(nt); m.normals.reserve(nn);
        m.face_v.reserve(3 * nf); m.face_t.reserve(3 * nf); m.face_n.reserve(3 * nf);
    }
    Cursor cur{p};
    while (cur.p < end) {
        if (cur.at('v')) {  // OBJ_loader.cpp:54-80
            ++cur.p;
            if (cur.at(' ')) m.vertices.push_back(cur.vec3());
            else if (cur.at('t')) { ++cur.p; m.texcoords.push_back(cur.vec3()); }
            else if (cur.at('n')) { ++cur.p; m.normals.push_back(cur.vec3()); }
        } else if (cur.at('f')) {  // OBJ_loader.cpp:81-149: first three index groups only
            ++cur.p;
            int32_t v[3] = {0, 0, 0}, t[3] = {0, 0, 0}, n[3] = {0, 0, 0};
            for (int k = 0; k < 3; ++k) {
                v[k] = cur.integer();
                if (cur.at('/')) {
                    ++cur.p;
                    if (cur.at('/')) { ++cur.p; n[k] = cur.integer(); }
                    else {
                        t[k] = cur.integer();
                        if (cur.at('/')) { ++cur.p; n[k] = cur.integer(); }
                    }
                }
            }
            for (int k = 0; k < 3; ++k) {
                m.face_v.push_back(v[k]);
                m.face_t.push_back(t[k]);
                m.face_n.push_back(n[k]);
            }
        }
        cur.to_next_line();
    }
}

template <class T>
void append(std::vector<T>& dst, const std::vector<T>& src) { dst.insert(dst.end(), src.begin(), src.end()); }

}  // namespace

int atr::parse_obj_text(const char* text, size_t len, HostMesh& m, int threads) {
    m = HostMesh();
    if (threads < 1) threads = 1;
    // Lines up to the last '\n' are parsed in place; a final line without one is copied with a
    // '\n' appended (OBJ_loader.cpp:329-330 gives the last chunk a closing '\n').
    size_t body = len;
    while (body > 0 && text[body - 1] != '\n') --body;
    const std::string tail = std::string(text + body, len - body) + "\n";
    // newline-aligned chunks of ~len / threads bytes (OBJ_loader.cpp:298-328)
    std::vector<std::pair<const char*, const char*>> chunks;
    const size_t step = std::max<size_t>(1, (body + size_t(threads) - 1) / size_t(threads));
    for (const char* p = text, *end = text + body; p < end;) {
        const char* q = p + std::min(step, size_t(end - p)) - 1;
        const void* nl = std::memchr(q, '\n', size_t(end - q));  // found: the body ends in '\n'
        q = static_cast<const char*>(nl);
        chunks.emplace_back(p, q + 1);
        p = q + 1;
    }
    if (len > body) chunks.emplace_back(tail.data(), tail.data() + tail.size());
    if (chunks.size() == 1) {
        parse_lines(chunks[0].first, chunks[0].second, m);
    } else if (chunks.size() > 1) {
        std::vector<HostMesh> part(chunks.size());
        std::vector<std::thread> pool;
        pool.reserve(chunks.size());
        for (size_t i = 0; i < chunks.size(); ++i)
            pool.emplace_back([&, i] { parse_lines(chunks[i].first, chunks[i].second, part[i]); });
        for (std::thread& t : pool) t.join();
        // join_chunks (OBJ_loader.cpp:190-227): in chunk order
        size_t nv = 0, nn = 0, nt = 0, nf = 0;
        for (const HostMesh& h : part) {
            nv += h.vertices.size(); nn += h.normals.size(); nt += h.texcoords.size(); nf += h.face_v.size();
        }
        m.vertices.reserve(nv); m.normals.reserve(nn); m.texcoords.reserve(nt);
        m.face_v.reserve(nf); m.face_t.reserve(nf); m.face_n.reserve(nf);
        for (const HostMesh& h : part) {
            append(m.vertices, h.vertices); append(m.normals, h.normals); append(m.texcoords, h.texcoords);
            append(m.face_v, h.face_v); append(m.face_t, h.face_t); append(m.face_n, h.face_n);
        }
    }
    // prep_model_data (OBJ_loader.cpp:229-267): relative indices, then drop the +1 offset
    const int32_t nv = int32_t(m.vertices.size()), nn = int32_t(m.normals.size()),
                  nt = int32_t(m.texcoords.size());
    for (size_t i = 0; i < m.face_v.size(); ++i) {
        if (m.face_t[i] < 0) m.face_t[i] += nt + 1;
        if (m.face_n[i] < 0) m.face_n[i] += nn + 1;
        if (m.face_v[i] < 0) m.face_v[i] += nv + 1;
        m.face_t[i] -= 1;
        m.face_v[i] -= 1;
        m.face_n[i] -= 1;
    }
    return ATR_OK;
}
