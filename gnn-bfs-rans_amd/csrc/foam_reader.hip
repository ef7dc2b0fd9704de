// OpenFOAM ASCII case reader, host code: the reference's
// OpenFOAMLoader (openfoam_loader.py:12-296) with its exact parsing rules --
// including its quirks, which define the graph the model was trained on:
//
//   labels (read_array, :53-65): the first "digits, blanks, '('" gives n; the
//     values are the digit runs of the WHOLE file from the 2nd on, n of them.
//     The header's digits (version, arch, note line) therefore shift the list
//     -- the "header-digit quirk" (n_cells 49,181 instead of 12,225 on the
//     reference case).
//   points (:25-46): every "(" [-0-9.eE+ whitespace]+ ")" group, split on
//     whitespace, float() of each token.
//   faces (:72-92): every digits [blanks] "(" [digits whitespace]+ ")" group.
//   scalar field (:114-142): n from "internalField nonuniform List<scalar> n";
//     values = the [-0-9.eE+]+ runs inside the first "(...)" after the first
//     "internalField", first n of them.
//   vector field (:144-189): line based (see mignn_foam_parse_vector_field).
//   cell centres (:191-227): per cell the SET of the vertices of its owner
//     faces, then its neighbour faces, averaged in the set's iteration order
//     (CPython's set: the order is emulated exactly so the float64 sums match
//     bit for bit).
//
// The caller passes the file bytes (no file I/O here) and output arrays of
// an upper-bound capacity; counts come back through *n_out.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <string>

#include "common.hpp"

namespace mignn {
namespace {

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_space(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v';
}
inline bool is_num_char(char c) {   // [-\d.eE+]
    return is_digit(c) || c == '-' || c == '.' || c == 'e' || c == 'E' || c == '+';
}

// re.search(r'(\d+)\s*\(') -> value of the digit run, or -1
int64_t first_count(const char* s, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        if (!is_digit(s[i])) continue;
        int64_t j = i;
        while (j < n && is_digit(s[j])) ++j;
        int64_t k = j;
        while (k < n && is_space(s[k])) ++k;
        if (k < n && s[k] == '(') return strtoll(std::string(s + i, s + j).c_str(), nullptr, 10);
        // a shorter suffix run ends at the same place: no match from inside it either
        i = j - 1;
    }
    return -1;
}

// float() of a token (Python accepts what strtod accepts for these tokens,
// surrounding whitespace excluded); false if not a full number
bool to_double(const char* b, const char* e, double* v) {
    std::string t(b, e);
    char* end = nullptr;
    *v = strtod(t.c_str(), &end);
    return end == t.c_str() + t.size() && !t.empty();
}

// CPython 3.x set of small non-negative ints (hash == value): insertion with
// linear probes + perturbation and table resizes, iteration in slot order
struct PySetEmu {
    std::vector<int64_t> table;   // -1 = empty
    size_t mask = 7, fill = 0, used = 0;
    PySetEmu() : table(8, -1) {}
    static constexpr int kLinearProbes = 9, kPerturbShift = 5;
    void insert_clean(std::vector<int64_t>& t, size_t m, int64_t key) {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & m;
        while (true) {
            if (t[i] < 0) { t[i] = key; return; }
            if (i + kLinearProbes <= m) {
                for (int j = 1; j <= kLinearProbes; ++j)
                    if (t[i + j] < 0) { t[i + j] = key; return; }
            }
            perturb >>= kPerturbShift;
            i = (i * 5 + 1 + perturb) & m;
        }
    }
    void resize(size_t minused) {
        size_t newsize = 8;
        while (newsize <= minused) newsize <<= 1;
        std::vector<int64_t> nt(newsize, -1);
        for (size_t s = 0; s <= mask; ++s)
            if (table[s] >= 0) insert_clean(nt, newsize - 1, table[s]);
        table.swap(nt);
        mask = newsize - 1;
        fill = used;
    }
    void add(int64_t key) {
        size_t perturb = static_cast<size_t>(key);
        size_t i = static_cast<size_t>(key) & mask;
        while (true) {
            size_t probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
            size_t k = i;
            while (true) {
                if (table[k] < 0) {   // unused slot (no dummies: nothing is deleted)
                    table[k] = key;
                    ++fill;
                    ++used;
                    if (fill * 5 >= mask * 3) resize(used > 50000 ? used * 2 : used * 4);
                    return;
                }
                if (table[k] == key) return;
                if (probes == 0) break;
                --probes;
                ++k;
            }
            perturb >>= kPerturbShift;
            i = (i * 5 + 1 + perturb) & mask;
        }
    }
};

// OpenFOAM's own list syntax: skip comments and the FoamFile { } dictionary,
// then "n ( v0 v1 ... )"; returns the offset of the count, or -1
int64_t body_start(const char* s, int64_t n) {
    int64_t i = 0;
    while (i < n) {
        if (s[i] == '/' && i + 1 < n && s[i + 1] == '*') {
            const char* e = strstr(s + i + 2, "*/");
            i = e ? (e - s) + 2 : n;
        } else if (s[i] == '/' && i + 1 < n && s[i + 1] == '/') {
            while (i < n && s[i] != '\n') ++i;
        } else if (strncmp(s + i, "FoamFile", 8) == 0) {
            const char* e = static_cast<const char*>(memchr(s + i, '}', n - i));
            i = e ? (e - s) + 1 : n;
        } else if (is_digit(s[i])) {
            return i;
        } else {
            ++i;
        }
    }
    return -1;
}

}  // namespace
}  // namespace mignn

using namespace mignn;

// compat 0 = the reference's read_array (:53-65, header-digit quirk);
// compat 1 = the list as OpenFOAM defines it (count after the header)
extern "C" int mignn_foam_parse_labels(const char* buf, int64_t len, int compat, int64_t* out,
                                       int64_t cap, int64_t* n_out) {
    MIGNN_REQUIRE(buf && n_out && (out || cap == 0), "foam_parse_labels: null pointer");
    if (compat == 1) {
        const int64_t b = body_start(buf, len);
        int64_t i = b, n = 0;
        while (b >= 0 && i < len && is_digit(buf[i])) n = n * 10 + (buf[i++] - '0');
        while (b >= 0 && i < len && is_space(buf[i])) ++i;
        if (b < 0 || i >= len || buf[i] != '(') {
            set_error("Could not find array size");
            return MIGNN_ERR_ARG;
        }
        if (n > cap) {
            set_error("foam_parse_labels: capacity %lld too small", (long long)cap);
            return MIGNN_ERR_SCRATCH;
        }
        int64_t got = 0;
        for (++i; i < len && got < n; ++i) {
            if (buf[i] == ')') break;
            if (!is_digit(buf[i])) continue;
            int64_t v = 0;
            while (i < len && is_digit(buf[i])) v = v * 10 + (buf[i++] - '0');
            out[got++] = v;
        }
        if (got != n) {
            set_error("foam_parse_labels: expected %lld labels, found %lld", (long long)n,
                      (long long)got);
            return MIGNN_ERR_ARG;
        }
        *n_out = got;
        return MIGNN_OK;
    }
    if (compat != 0) {
        set_error("foam_parse_labels: compat must be 0 or 1");
        return MIGNN_ERR_ARG;
    }
    const int64_t n = first_count(buf, len);
    if (n < 0) {
        set_error("Could not find array size");
        return MIGNN_ERR_ARG;
    }
    int64_t runs = 0, got = 0;
    for (int64_t i = 0; i < len && got < n; ++i) {
        if (!is_digit(buf[i])) continue;
        int64_t j = i;
        int64_t v = 0;
        while (j < len && is_digit(buf[j])) v = v * 10 + (buf[j++] - '0');
        if (runs++ >= 1) {   // matches[1 : n + 1]
            if (got >= cap) {
                set_error("foam_parse_labels: capacity %lld too small", (long long)cap);
                return MIGNN_ERR_SCRATCH;
            }
            out[got++] = v;
        }
        i = j - 1;
    }
    *n_out = got;
    return MIGNN_OK;
}

extern "C" int mignn_foam_parse_points(const char* buf, int64_t len, double* out, int64_t cap_rows,
                                       int64_t* n_rows) {
    MIGNN_REQUIRE(buf && n_rows && (out || cap_rows == 0), "foam_parse_points: null pointer");
    if (first_count(buf, len) < 0) {
        set_error("Could not find number of points");
        return MIGNN_ERR_ARG;
    }
    int64_t rows = 0;
    for (int64_t i = 0; i < len; ++i) {
        if (buf[i] != '(') continue;
        int64_t j = i + 1;
        while (j < len && (is_num_char(buf[j]) || is_space(buf[j]))) ++j;
        if (j == i + 1 || j >= len || buf[j] != ')') continue;
        double v[3];
        int nv = 0;
        for (int64_t k = i + 1; k < j;) {
            while (k < j && is_space(buf[k])) ++k;
            int64_t e = k;
            while (e < j && !is_space(buf[e])) ++e;
            if (e > k) {
                double d;
                if (!to_double(buf + k, buf + e, &d)) {
                    set_error("could not convert string to float: '%.*s'", (int)(e - k), buf + k);
                    return MIGNN_ERR_ARG;
                }
                if (nv < 3) v[nv] = d;
                ++nv;
            }
            k = e;
        }
        if (nv != 3) {
            set_error("foam_parse_points: a point with %d coordinates", nv);
            return MIGNN_ERR_ARG;
        }
        if (rows >= cap_rows) {
            set_error("foam_parse_points: capacity too small");
            return MIGNN_ERR_SCRATCH;
        }
        memcpy(out + 3 * rows, v, sizeof(v));
        ++rows;
        i = j;
    }
    *n_rows = rows;
    return MIGNN_OK;
}

// faces as CSR: offsets[n_faces + 1], verts[]
extern "C" int mignn_foam_parse_faces(const char* buf, int64_t len, int64_t* offsets,
                                      int64_t cap_faces, int64_t* verts, int64_t cap_verts,
                                      int64_t* n_faces, int64_t* n_verts) {
    MIGNN_REQUIRE(buf && offsets && verts && n_faces && n_verts, "foam_parse_faces: null pointer");
    if (first_count(buf, len) < 0) {
        set_error("Could not find number of faces");
        return MIGNN_ERR_ARG;
    }
    int64_t nf = 0, nv = 0;
    offsets[0] = 0;
    for (int64_t i = 0; i < len; ++i) {
        if (!is_digit(buf[i])) continue;
        int64_t j = i;
        while (j < len && is_digit(buf[j])) ++j;
        int64_t k = j;
        while (k < len && is_space(buf[k])) ++k;
        if (k < len && buf[k] == '(') {
            int64_t e = k + 1;
            while (e < len && (is_digit(buf[e]) || is_space(buf[e]))) ++e;
            if (e > k + 1 && e < len && buf[e] == ')') {
                if (nf + 1 > cap_faces) {
                    set_error("foam_parse_faces: face capacity too small");
                    return MIGNN_ERR_SCRATCH;
                }
                for (int64_t p = k + 1; p < e;) {
                    while (p < e && is_space(buf[p])) ++p;
                    if (p >= e) break;
                    int64_t v = 0;
                    while (p < e && is_digit(buf[p])) v = v * 10 + (buf[p++] - '0');
                    if (nv >= cap_verts) {
                        set_error("foam_parse_faces: vertex capacity too small");
                        return MIGNN_ERR_SCRATCH;
                    }
                    verts[nv++] = v;
                }
                offsets[++nf] = nv;
                i = e;   // findall resumes after the match
                continue;
            }
        }
        i = j - 1;
    }
    *n_faces = nf;
    *n_verts = nv;
    return MIGNN_OK;
}

extern "C" int mignn_foam_parse_scalar_field(const char* buf, int64_t len, double* out, int64_t cap,
                                             int64_t* n_out) {
    MIGNN_REQUIRE(buf && n_out && (out || cap == 0), "foam_parse_scalar_field: null pointer");
    // n: internalField\s+nonuniform\s+List<scalar>\s*(\d+)
    const char* key = "internalField";
    const size_t kl = strlen(key);
    int64_t n = -1;
    for (const char* p = strstr(buf, key); p && p < buf + len; p = strstr(p + 1, key)) {
        const char* q = p + kl;
        const char* e = buf + len;
        const char* r = q;
        while (r < e && is_space(*r)) ++r;
        if (r == q || strncmp(r, "nonuniform", 10) != 0) continue;
        q = r + 10;
        r = q;
        while (r < e && is_space(*r)) ++r;
        if (r == q || strncmp(r, "List<scalar>", 12) != 0) continue;
        r += 12;
        while (r < e && is_space(*r)) ++r;
        if (r < e && is_digit(*r)) {
            n = strtoll(r, nullptr, 10);
            break;
        }
    }
    if (n < 0) {
        set_error("Could not find internal field");
        return MIGNN_ERR_ARG;
    }
    // values: internalField[^(]*\(([^)]+)\) -- the first internalField, next '(' ... ')'
    const char* p = strstr(buf, key);
    const char* e = buf + len;
    const char* op = p ? static_cast<const char*>(memchr(p, '(', e - p)) : nullptr;
    const char* cp = op ? static_cast<const char*>(memchr(op + 1, ')', e - op - 1)) : nullptr;
    if (!op || !cp || cp == op + 1) {
        set_error("Could not find values");
        return MIGNN_ERR_ARG;
    }
    int64_t got = 0;
    for (const char* k = op + 1; k < cp && got < n;) {
        if (!is_num_char(*k)) {
            ++k;
            continue;
        }
        const char* t = k;
        while (t < cp && is_num_char(*t)) ++t;
        double d;
        if (!to_double(k, t, &d)) {
            set_error("could not convert string to float: '%.*s'", (int)(t - k), k);
            return MIGNN_ERR_ARG;
        }
        if (got >= cap) {
            set_error("foam_parse_scalar_field: capacity too small");
            return MIGNN_ERR_SCRATCH;
        }
        out[got++] = d;
        k = t;
    }
    *n_out = got;
    return MIGNN_OK;
}

// read_vector_field (:144-189): the first line containing "internalField" and
// "nonuniform"; n = first digit run of the next line; the list starts after
// the first of the next 4 lines containing '('; then per line the first
// "(" [-0-9.eE+ whitespace]+ ")" group with exactly 3 numbers, until n.
extern "C" int mignn_foam_parse_vector_field(const char* buf, int64_t len, double* out,
                                             int64_t cap_rows, int64_t* n_rows) {
    MIGNN_REQUIRE(buf && n_rows && (out || cap_rows == 0), "foam_parse_vector_field: null pointer");
    std::vector<std::pair<int64_t, int64_t>> lines;   // [begin, end) incl. newline
    for (int64_t b = 0; b < len;) {
        int64_t e = b;
        while (e < len && buf[e] != '\n') ++e;
        lines.push_back({b, e < len ? e + 1 : e});
        b = e + 1;
    }
    auto contains = [&](size_t li, const char* s) {
        const std::string l(buf + lines[li].first, buf + lines[li].second);
        return l.find(s) != std::string::npos;
    };
    int64_t n = -1;
    size_t start = 0;
    bool found = false;
    for (size_t i = 0; i < lines.size(); ++i) {
        if (contains(i, "internalField") && contains(i, "nonuniform")) {
            if (i + 1 < lines.size()) {
                for (int64_t k = lines[i + 1].first; k < lines[i + 1].second; ++k)
                    if (is_digit(buf[k])) {
                        n = strtoll(buf + k, nullptr, 10);
                        break;
                    }
            }
            for (size_t j = i + 1; j < lines.size() && j < i + 5; ++j)
                if (contains(j, "(")) {
                    start = j + 1;
                    found = true;
                    break;
                }
            break;
        }
    }
    if (n < 0 || !found) {
        set_error("Could not find internal field");
        return MIGNN_ERR_ARG;
    }
    int64_t rows = 0;
    for (size_t i = start; i < lines.size() && rows < n; ++i) {
        const char* b = buf + lines[i].first;
        const char* e = buf + lines[i].second;
        for (const char* p = b; p < e; ++p) {   // first matching group of the line
            if (*p != '(') continue;
            const char* q = p + 1;
            while (q < e && (is_num_char(*q) || is_space(*q))) ++q;
            if (q == p + 1 || q >= e || *q != ')') continue;
            double v[3];
            int nv = 0;
            bool ok = true;
            for (const char* k = p + 1; k < q;) {
                while (k < q && is_space(*k)) ++k;
                const char* t = k;
                while (t < q && !is_space(*t)) ++t;
                if (t > k) {
                    double d;
                    if (!to_double(k, t, &d)) ok = false;
                    if (nv < 3) v[nv] = d;
                    ++nv;
                }
                k = t;
            }
            if (!ok) {
                set_error("could not convert a vector component to float");
                return MIGNN_ERR_ARG;
            }
            if (nv == 3) {
                if (rows >= cap_rows) {
                    set_error("foam_parse_vector_field: capacity too small");
                    return MIGNN_ERR_SCRATCH;
                }
                memcpy(out + 3 * rows, v, sizeof(v));
                ++rows;
            }
            break;
        }
    }
    if (rows != n) {
        set_error("Expected %lld vectors, found %lld", (long long)n, (long long)rows);
        return MIGNN_ERR_ARG;
    }
    *n_rows = rows;
    return MIGNN_OK;
}

// get_cell_centers (:191-227)
extern "C" int mignn_foam_cell_centers(const double* points, int64_t n_points,
                                       const int64_t* owner, int64_t n_owner,
                                       const int64_t* neighbour, int64_t n_neighbour,
                                       const int64_t* face_off, const int64_t* face_verts,
                                       int64_t n_faces, int64_t n_cells, double* centers) {
    MIGNN_REQUIRE(points && owner && face_off && face_verts && centers &&
                      (neighbour || n_neighbour == 0),
                  "foam_cell_centers: null pointer");
    // faces of each cell: its owner faces (face order), then its neighbour faces
    std::vector<int64_t> cnt(n_cells + 1, 0);
    for (int64_t i = 0; i < n_owner; ++i) cnt[owner[i] + 1]++;
    for (int64_t i = 0; i < n_neighbour; ++i) cnt[neighbour[i] + 1]++;
    for (int64_t c = 0; c < n_cells; ++c) cnt[c + 1] += cnt[c];
    std::vector<int64_t> at(cnt.begin(), cnt.end() - 1), cf(cnt[n_cells]);
    for (int64_t i = 0; i < n_owner; ++i) {
        if (owner[i] < 0 || owner[i] >= n_cells || i >= n_faces) {
            set_error("foam_cell_centers: face %lld / cell %lld out of range", (long long)i,
                      (long long)owner[i]);
            return MIGNN_ERR_ARG;
        }
        cf[at[owner[i]]++] = i;
    }
    for (int64_t i = 0; i < n_neighbour; ++i) {
        if (neighbour[i] < 0 || neighbour[i] >= n_cells || i >= n_faces) {
            set_error("foam_cell_centers: neighbour face %lld out of range", (long long)i);
            return MIGNN_ERR_ARG;
        }
        cf[at[neighbour[i]]++] = i;
    }
    for (int64_t c = 0; c < n_cells; ++c) {
        double* o = centers + 3 * c;
        if (cnt[c + 1] == cnt[c]) {
            o[0] = o[1] = o[2] = 0.0;
            continue;
        }
        PySetEmu set;
        for (int64_t t = cnt[c]; t < cnt[c + 1]; ++t) {
            const int64_t f = cf[t];
            for (int64_t v = face_off[f]; v < face_off[f + 1]; ++v) set.add(face_verts[v]);
        }
        // np.mean(points[list(set)], axis=0): a sequential add.reduce over the
        // rows in set order, starting from the first row, then / m
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        int64_t m = 0;
        for (size_t k = 0; k <= set.mask; ++k) {
            const int64_t p = set.table[k];
            if (p < 0) continue;
            if (p >= n_points) {
                set_error("foam_cell_centers: vertex %lld out of range", (long long)p);
                return MIGNN_ERR_ARG;
            }
            if (m == 0) {
                s0 = points[3 * p];
                s1 = points[3 * p + 1];
                s2 = points[3 * p + 2];
            } else {
                s0 += points[3 * p];
                s1 += points[3 * p + 1];
                s2 += points[3 * p + 2];
            }
            ++m;
        }
        o[0] = s0 / static_cast<double>(m);
        o[1] = s1 / static_cast<double>(m);
        o[2] = s2 / static_cast<double>(m);
    }
    return MIGNN_OK;
}
