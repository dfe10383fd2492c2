// arx_io.cpp -- native readers for the reference's input formats (host code of libarx.so).
//
// The reference reads its inputs with three third-party libraries vendored in its tree; the
// behaviour that reaches the IR path is restated here (not copied) and pinned against the
// reference's own compiled code by tests/golden fixtures (oracle/refdriver/refdump.cpp):
//   * OBJ/MTL  -- tinyobj v2.0.0 (R/prebuild/common/3rdParty/tiny_obj_loader.h):
//     line reader (\n, \r, \r\n), number parser (digit-wise mantissa, pow(5,e)*2^e
//     exponent, :805-936), face index fixing (:739-760), usemtl / o / g shape flushing
//     (:2336-2487), ear-clipping triangulation (:1357-1580), mtllib search (:2047-2073),
//     LoadMtl material list incl. the always-flushed last material (:1669-2041);
//     then OptixModel::loadOBJ's per-(shape, material) split with (v,n,t) vertex dedup
//     (R/prebuild/obj_raytracer/OptixModel.cpp:37-151).
//   * WAV      -- AudioFile<float>::decodeWaveFile (OR/AudioFile.h:502-640): RIFF chunk
//     walk, PCM 8/16/24/32 and IEEE float 32, sample scaling of :1242-1269.
//   * config   -- cJSON 1.7.16 value semantics (case-insensitive keys, strtod numbers) +
//     Context::loadContext defaults and rounding (OR/Context.cpp:15-164).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/arx.h"

void arx_set_last_error(const std::string& m);  // arx_capi.cpp

namespace {

arx_status io_fail(arx_status s, const std::string& m) {
    arx_set_last_error(m);
    return s;
}

// ------------------------------------------------------------------ OBJ ----
struct Corner {
    int v = -1, n = -1, t = -1;
};

struct ObjShape {
    std::string name;
    std::vector<Corner> corners;   // 3 per triangle
    std::vector<int> material_ids; // per triangle
};

struct ObjData {
    std::vector<float> v;  // positions
    std::vector<ObjShape> shapes;
    std::vector<std::string> materials;
};

bool is_space(char c) { return c == ' ' || c == '\t'; }
bool is_new_line(char c) { return c == '\r' || c == '\n' || c == '\0'; }
bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }

// Reads one line; accepts \n, \r and \r\n endings.  Returns false at end of input.
bool next_line(const std::string& data, size_t& pos, std::string& line) {
    if (pos >= data.size()) return false;
    line.clear();
    while (pos < data.size()) {
        const char c = data[pos++];
        if (c == '\n') return true;
        if (c == '\r') {
            if (pos < data.size() && data[pos] == '\n') ++pos;
            return true;
        }
        line.push_back(c);
    }
    return true;
}

// Number grammar and arithmetic of tinyobj's tryParseDouble: integer digits accumulated as
// m = m*10 + d, fraction digits added as d * 10^-k (table up to k = 7, pow beyond), exponent
// applied as ldexp(m * 5^e, e).
bool parse_double(const char* s, const char* end, double* out) {
    if (s >= end) return false;
    double mant = 0.0;
    int expo = 0;
    char sign = '+', esign = '+';
    const char* c = s;
    int read = 0;
    bool more = false;
    bool lead_dot = false;
    if (*c == '+' || *c == '-') {
        sign = *c;
        ++c;
        if (c != end && *c == '.') lead_dot = true;
    } else if (is_digit(*c)) {
    } else if (*c == '.') {
        lead_dot = true;
    } else {
        return false;
    }
    more = (c != end);
    if (!lead_dot) {
        while (more && is_digit(*c)) {
            mant *= 10;
            mant += (int)(*c - '0');
            ++c;
            ++read;
            more = (c != end);
        }
        if (read == 0) return false;
    }
    if (more) {
        if (*c == '.') {
            ++c;
            read = 1;
            more = (c != end);
            static const double tab[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (more && is_digit(*c)) {
                mant += (int)(*c - '0') * (read < 8 ? tab[read] : std::pow(10.0, -read));
                ++read;
                ++c;
                more = (c != end);
            }
        } else if (*c == 'e' || *c == 'E') {
        } else {
            more = false;  // assemble
            goto assemble;
        }
        if (more && (*c == 'e' || *c == 'E')) {
            ++c;
            more = (c != end);
            if (more && (*c == '+' || *c == '-')) {
                esign = *c;
                ++c;
            } else if (is_digit(*c)) {
            } else {
                return false;
            }
            read = 0;
            more = (c != end);
            while (more && is_digit(*c)) {
                expo *= 10;
                expo += (int)(*c - '0');
                ++c;
                ++read;
                more = (c != end);
            }
            expo *= (esign == '+' ? 1 : -1);
            if (read == 0) return false;
        }
    }
assemble:
    *out = (sign == '+' ? 1 : -1) * (expo ? std::ldexp(mant * std::pow(5.0, expo), expo) : mant);
    return true;
}

// tinyobj parseReal: skip blanks, parse up to the next blank / CR, fall back to default.
float parse_real(const char** tok, double def) {
    *tok += std::strspn(*tok, " \t");
    const char* end = *tok + std::strcspn(*tok, " \t\r");
    double v = def;
    parse_double(*tok, end, &v);
    *tok = end;
    return (float)v;
}

bool fix_index(int idx, int n, int* ret) {
    if (idx > 0) {
        *ret = idx - 1;
        return true;
    }
    if (idx == 0) return false;
    *ret = n + idx;  // negative = relative
    return true;
}

// "i", "i/j", "i//k", "i/j/k"
bool parse_corner(const char** tok, int vs, int ns, int ts, Corner* out) {
    Corner c;
    if (!fix_index(std::atoi(*tok), vs, &c.v)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') {
        *out = c;
        return true;
    }
    ++*tok;
    if ((*tok)[0] == '/') {
        ++*tok;
        if (!fix_index(std::atoi(*tok), ns, &c.n)) return false;
        *tok += std::strcspn(*tok, "/ \t\r");
        *out = c;
        return true;
    }
    if (!fix_index(std::atoi(*tok), ts, &c.t)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') {
        *out = c;
        return true;
    }
    ++*tok;
    if (!fix_index(std::atoi(*tok), ns, &c.n)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    *out = c;
    return true;
}

// point-in-polygon crossing test (W. R. Franklin's pnpoly), float arithmetic
int pnpoly3(const float* vx, const float* vy, float tx, float ty) {
    int c = 0;
    for (int i = 0, j = 2; i < 3; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i]))
            c = !c;
    }
    return c;
}

struct Pending {
    std::vector<std::vector<Corner>> faces;
    bool lines_or_points = false;
    bool empty() const { return faces.empty() && !lines_or_points; }
};

// Ear-clipping triangulation of one face into shape (tinyobj's algorithm with triangulate=true).
void triangulate_face(const std::vector<Corner>& face, const std::vector<float>& v, int material, ObjShape& shape) {
    size_t np = face.size();
    if (np < 3) return;
    auto vx = [&](int idx, int ax) -> float { return v[(size_t)idx * 3 + ax]; };
    auto valid = [&](int idx, int ax) { return idx >= 0 && (size_t)idx * 3 + ax < v.size(); };
    // choose the projection plane from the first non-degenerate corner
    size_t axes[2] = {1, 2};
    for (size_t k = 0; k < np; ++k) {
        const int i0 = face[(k + 0) % np].v, i1 = face[(k + 1) % np].v, i2 = face[(k + 2) % np].v;
        if (!valid(i0, 2) || !valid(i1, 2) || !valid(i2, 2)) continue;
        const float e0x = vx(i1, 0) - vx(i0, 0), e0y = vx(i1, 1) - vx(i0, 1), e0z = vx(i1, 2) - vx(i0, 2);
        const float e1x = vx(i2, 0) - vx(i1, 0), e1y = vx(i2, 1) - vx(i1, 1), e1z = vx(i2, 2) - vx(i1, 2);
        const float cx = std::fabs(e0y * e1z - e0z * e1y);
        const float cy = std::fabs(e0z * e1x - e0x * e1z);
        const float cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = 1.1920929e-07f;  // numeric_limits<float>::epsilon
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) {
                axes[0] = 0;
                if (cz > cx && cz > cy) axes[1] = 1;
            }
            break;
        }
    }
    float area = 0.0f;
    for (size_t k = 0; k < np; ++k) {
        const int i0 = face[(k + 0) % np].v, i1 = face[(k + 1) % np].v;
        if (!valid(i0, (int)axes[0]) || !valid(i0, (int)axes[1]) || !valid(i1, (int)axes[0]) ||
            !valid(i1, (int)axes[1]))
            continue;
        const float v0x = vx(i0, (int)axes[0]), v0y = vx(i0, (int)axes[1]);
        const float v1x = vx(i1, (int)axes[0]), v1y = vx(i1, (int)axes[1]);
        area += (v0x * v1y - v0y * v1x) * 0.5f;
    }
    std::vector<Corner> rem = face;
    size_t guess = 0;
    size_t iterations = face.size();
    size_t prev_count = rem.size();
    Corner ind[3];
    float px[3], py[3];
    while (rem.size() > 3 && iterations > 0) {
        np = rem.size();
        if (guess >= np) guess -= np;
        if (prev_count != np) {
            prev_count = np;
            iterations = np;
        } else {
            --iterations;
        }
        for (int k = 0; k < 3; ++k) {
            ind[k] = rem[(guess + k) % np];
            if (!valid(ind[k].v, (int)axes[0]) || !valid(ind[k].v, (int)axes[1])) {
                px[k] = 0.0f;
                py[k] = 0.0f;
            } else {
                px[k] = vx(ind[k].v, (int)axes[0]);
                py[k] = vx(ind[k].v, (int)axes[1]);
            }
        }
        const float e0x = px[1] - px[0], e0y = py[1] - py[0];
        const float e1x = px[2] - px[1], e1y = py[2] - py[1];
        const float cross = e0x * e1y - e0y * e1x;
        if (cross * area < 0.0f) {  // reflex corner
            guess += 1;
            continue;
        }
        bool overlap = false;
        for (size_t other = 3; other < np; ++other) {
            const size_t idx = (guess + other) % np;
            if (idx >= rem.size()) continue;
            const int ov = rem[idx].v;
            if (!valid(ov, (int)axes[0]) || !valid(ov, (int)axes[1])) continue;
            if (pnpoly3(px, py, vx(ov, (int)axes[0]), vx(ov, (int)axes[1]))) {
                overlap = true;
                break;
            }
        }
        if (overlap) {
            guess += 1;
            continue;
        }
        for (int k = 0; k < 3; ++k) shape.corners.push_back(ind[k]);
        shape.material_ids.push_back(material);
        size_t rm = (guess + 1) % np;  // drop the ear's middle corner
        rem.erase(rem.begin() + (ptrdiff_t)rm);
    }
    if (rem.size() == 3) {
        for (int k = 0; k < 3; ++k) shape.corners.push_back(rem[k]);
        shape.material_ids.push_back(material);
    }
}

// exportGroupsToShape: false when nothing is pending.
bool flush_group(ObjShape& shape, const Pending& p, int material, const std::string& name, const std::vector<float>& v) {
    if (p.empty()) return false;
    shape.name = name;
    for (const auto& f : p.faces) triangulate_face(f, v, material, shape);
    return true;
}

void load_mtl_text(const std::string& text, std::vector<std::string>& mats, std::map<std::string, int>& map) {
    std::string cur;  // the default material has an empty name
    size_t pos = 0;
    std::string line;
    while (next_line(text, pos, line)) {
        const size_t last = line.find_last_not_of(" \t");
        line = (last == std::string::npos) ? std::string() : line.substr(0, last + 1);
        if (line.empty()) continue;
        const char* tok = line.c_str();
        tok += std::strspn(tok, " \t");
        if (tok[0] == '\0' || tok[0] == '#') continue;
        if (std::strncmp(tok, "newmtl", 6) == 0 && is_space(tok[6])) {
            if (!cur.empty()) {
                map.insert({cur, (int)mats.size()});
                mats.push_back(cur);
            }
            cur = std::string(tok + 7);
        }
    }
    map.insert({cur, (int)mats.size()});  // the last material is always flushed
    mats.push_back(cur);
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

arx_status parse_obj(const std::string& path, const std::string& mtl_dir_in, ObjData& out) {
    std::string text;
    if (!read_file(path, text)) return io_fail(ARX_ERR_IO, "Cannot open file [" + path + "]");
    std::string mtl_dir = mtl_dir_in;
    if (!mtl_dir.empty() && mtl_dir.back() != '/') mtl_dir += '/';
    std::vector<float> vn_count_dummy;
    size_t n_vn = 0, n_vt = 0;
    std::map<std::string, int> mat_map;
    int material = -1;
    std::string name;
    ObjShape shape;
    Pending pend;
    size_t pos = 0;
    std::string line;
    while (next_line(text, pos, line)) {
        if (line.empty()) continue;
        const char* tok = line.c_str();
        tok += std::strspn(tok, " \t");
        if (tok[0] == '\0' || tok[0] == '#') continue;
        if (tok[0] == 'v' && is_space(tok[1])) {
            tok += 2;
            const float x = parse_real(&tok, 0.0), y = parse_real(&tok, 0.0), z = parse_real(&tok, 0.0);
            out.v.push_back(x);
            out.v.push_back(y);
            out.v.push_back(z);
            continue;
        }
        if (tok[0] == 'v' && tok[1] == 'n' && is_space(tok[2])) {
            ++n_vn;
            continue;
        }
        if (tok[0] == 'v' && tok[1] == 't' && is_space(tok[2])) {
            ++n_vt;
            continue;
        }
        if ((tok[0] == 'l' || tok[0] == 'p') && is_space(tok[1])) {
            tok += 2;
            while (!is_new_line(tok[0])) {
                Corner c;
                if (!parse_corner(&tok, (int)(out.v.size() / 3), (int)n_vn, (int)n_vt, &c))
                    return io_fail(ARX_ERR_IO, "bad line/point index in " + path);
                tok += std::strspn(tok, " \t\r");
            }
            pend.lines_or_points = true;
            continue;
        }
        if (tok[0] == 'f' && is_space(tok[1])) {
            tok += 2;
            tok += std::strspn(tok, " \t");
            std::vector<Corner> face;
            while (!is_new_line(tok[0])) {
                Corner c;
                if (!parse_corner(&tok, (int)(out.v.size() / 3), (int)n_vn, (int)n_vt, &c))
                    return io_fail(ARX_ERR_IO, "Failed parse `f' line (e.g. zero value for face index) in " + path);
                face.push_back(c);
                tok += std::strspn(tok, " \t\r");
            }
            pend.faces.push_back(face);
            continue;
        }
        if (std::strncmp(tok, "usemtl", 6) == 0 && is_space(tok[6])) {
            const std::string mname(tok + 7);
            int id = -1;
            auto it = mat_map.find(mname);
            if (it != mat_map.end()) id = it->second;
            if (id != material) {
                flush_group(shape, pend, material, name, out.v);
                pend.faces.clear();
                material = id;
            }
            continue;
        }
        if (std::strncmp(tok, "mtllib", 6) == 0 && is_space(tok[6])) {
            std::stringstream ss(std::string(tok + 7));
            std::string fn;
            while (std::getline(ss, fn, ' ')) {
                std::string mtext;
                if (read_file(mtl_dir + fn, mtext)) {
                    load_mtl_text(mtext, out.materials, mat_map);
                    break;
                }
            }
            continue;
        }
        if (tok[0] == 'g' && is_space(tok[1])) {
            flush_group(shape, pend, material, name, out.v);
            if (!shape.corners.empty()) out.shapes.push_back(shape);
            shape = ObjShape();
            pend = Pending();
            // group name = tokens after 'g' joined by ' ' (names[1..])
            std::vector<std::string> names;
            while (!is_new_line(tok[0])) {
                tok += std::strspn(tok, " \t");
                const size_t e = std::strcspn(tok, " \t\r");
                names.emplace_back(tok, e);
                tok += e;
                tok += std::strspn(tok, " \t\r");
            }
            if (names.size() >= 2) {
                std::string n = names[1];
                for (size_t i = 2; i < names.size(); ++i) n += " " + names[i];
                name = n;
            }
            continue;
        }
        if (tok[0] == 'o' && is_space(tok[1])) {
            if (flush_group(shape, pend, material, name, out.v)) out.shapes.push_back(shape);
            pend = Pending();
            shape = ObjShape();
            name = std::string(tok + 2);
            continue;
        }
    }
    const bool ret = flush_group(shape, pend, material, name, out.v);
    if (ret || !shape.corners.empty()) out.shapes.push_back(shape);
    return ARX_OK;
}

}  // namespace

// Loaded model: one mesh per (shape, material) as OptixModel::loadOBJ builds them.
struct arx_model {
    struct MeshOut {
        std::string name;
        std::vector<float> v;
        std::vector<int32_t> idx;
    };
    std::vector<MeshOut> meshes;
    int64_t n_materials = 0;
    int64_t n_shapes = 0;
    int64_t n_positions = 0;
};

namespace {

struct CornerKey {
    int v, n, t;
    bool operator<(const CornerKey& o) const {
        if (v != o.v) return v < o.v;
        if (n != o.n) return n < o.n;
        return t < o.t;
    }
};

// OptixModel.cpp:104-141 (loadOBJ) / :240-274 (place_receiver_half uses shapes[0] only).
void split_meshes(const ObjData& d, bool first_shape_only, const char* forced_name, arx_model& m) {
    for (const auto& sh : d.shapes) {
        std::set<int> ids(sh.material_ids.begin(), sh.material_ids.end());
        for (int mid : ids) {
            arx_model::MeshOut mesh;
            std::map<CornerKey, int> known;
            for (size_t f = 0; f < sh.material_ids.size(); ++f) {
                if (sh.material_ids[f] != mid) continue;
                for (int k = 0; k < 3; ++k) {
                    const Corner& c = sh.corners[3 * f + k];
                    const CornerKey key{c.v, c.n, c.t};
                    auto it = known.find(key);
                    int id;
                    if (it != known.end()) {
                        id = it->second;
                    } else {
                        id = (int)(mesh.v.size() / 3);
                        known[key] = id;
                        for (int a = 0; a < 3; ++a) mesh.v.push_back(d.v[(size_t)c.v * 3 + a]);
                    }
                    mesh.idx.push_back(id);
                }
                if (forced_name)
                    mesh.name = forced_name;
                else if (mid >= 0)
                    mesh.name = d.materials[(size_t)mid];
            }
            if (!mesh.v.empty()) m.meshes.push_back(mesh);
        }
        if (first_shape_only) break;
    }
}

}  // namespace

extern "C" {

arx_status arx_model_load_obj(const char* path, const char* mtl_dir, int first_shape_only, const char* forced_name,
                              arx_model** out) {
    if (!path || !out) return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = nullptr;
    const std::string p(path);
    // loadOBJ: mtlDir = objFile.substr(0, rfind('/') + 1) (OptixModel.cpp:79)
    const std::string dir = mtl_dir ? std::string(mtl_dir) : p.substr(0, p.rfind('/') + 1);
    ObjData d;
    arx_status st = parse_obj(p, dir, d);
    if (st != ARX_OK) return st;
    // loadOBJ / HalfSphere throw "could not parse materials ..." without an MTL
    if (d.materials.empty()) return io_fail(ARX_ERR_IO, "could not parse materials ... (" + p + ")");
    // addVertex indexes attributes.vertices unchecked; out-of-range corners are rejected here
    for (const auto& sh : d.shapes)
        for (const auto& c : sh.corners)
            if (c.v < 0 || (size_t)c.v >= d.v.size() / 3)
                return io_fail(ARX_ERR_IO, "vertex index out of range in " + p);
    arx_model* m = new arx_model();
    m->n_materials = (int64_t)d.materials.size();
    m->n_shapes = (int64_t)d.shapes.size();
    m->n_positions = (int64_t)(d.v.size() / 3);
    split_meshes(d, first_shape_only != 0, forced_name, *m);
    *out = m;
    return ARX_OK;
}

void arx_model_free(arx_model* m) { delete m; }

int64_t arx_model_mesh_count(const arx_model* m) { return m ? (int64_t)m->meshes.size() : 0; }

int64_t arx_model_material_count(const arx_model* m) { return m ? m->n_materials : 0; }

void arx_model_info(const arx_model* m, int64_t* n_shapes, int64_t* n_materials, int64_t* n_positions) {
    if (n_shapes) *n_shapes = m ? m->n_shapes : 0;
    if (n_materials) *n_materials = m ? m->n_materials : 0;
    if (n_positions) *n_positions = m ? m->n_positions : 0;
}

int64_t arx_model_triangle_count(const arx_model* m) {
    int64_t n = 0;
    if (m)
        for (const auto& me : m->meshes) n += (int64_t)(me.idx.size() / 3);
    return n;
}

// Flattens the meshes in model order into the triangle soup arx_set_scene takes, each
// triangle carrying getMaterialAbsorption(mesh name) (AudioRenderer.cpp:34-56, :455).
arx_status arx_model_flatten(const arx_model* m, const char* const* names, const float* absorption,
                             size_t n_materials, float* tri_vertices, float* tri_absorption) {
    if (!m || !tri_vertices || (n_materials && (!names || !absorption)))
        return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    int64_t t = 0;
    for (const auto& me : m->meshes) {
        const float a = arx_material_absorption(me.name.c_str(), names, absorption, n_materials);
        for (size_t f = 0; f < me.idx.size() / 3; ++f, ++t) {
            for (int k = 0; k < 3; ++k)
                for (int ax = 0; ax < 3; ++ax)
                    tri_vertices[t * 9 + k * 3 + ax] = me.v[(size_t)me.idx[3 * f + k] * 3 + ax];
            if (tri_absorption) tri_absorption[t] = a;
        }
    }
    return ARX_OK;
}

arx_status arx_model_mesh(const arx_model* m, int64_t i, const char** name, const float** vertices,
                          int64_t* n_vertices, const int32_t** indices, int64_t* n_triangles) {
    if (!m || i < 0 || i >= (int64_t)m->meshes.size()) return io_fail(ARX_ERR_INVALID_ARGUMENT, "bad mesh index");
    const auto& me = m->meshes[(size_t)i];
    if (name) *name = me.name.c_str();
    if (vertices) *vertices = me.v.data();
    if (n_vertices) *n_vertices = (int64_t)(me.v.size() / 3);
    if (indices) *indices = me.idx.data();
    if (n_triangles) *n_triangles = (int64_t)(me.idx.size() / 3);
    return ARX_OK;
}

// ------------------------------------------------------------------ WAV ----
arx_status arx_wav_load(const char* path, float** samples, int32_t* channels, int64_t* frames, int32_t* sample_rate,
                        int32_t* bit_depth) {
    if (!path || !samples || !channels || !frames || !sample_rate)
        return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    *samples = nullptr;
    std::string s;
    if (!read_file(path, s)) return io_fail(ARX_ERR_IO, std::string("cannot open ") + path);
    const std::vector<uint8_t> d(s.begin(), s.end());
    auto u16 = [&](size_t i) -> int16_t { return (int16_t)((d[i + 1] << 8) | d[i]); };
    auto u32 = [&](size_t i) -> int32_t {
        return (int32_t)(((uint32_t)d[i + 3] << 24) | ((uint32_t)d[i + 2] << 16) | ((uint32_t)d[i + 1] << 8) | d[i]);
    };
    auto chunk = [&](const char* id, size_t start) -> int64_t {
        int64_t i = (int64_t)start;
        while (d.size() >= 4 && (size_t)i < d.size() - 4) {
            if (std::memcmp(&d[(size_t)i], id, 4) == 0) return i;
            i += 4;
            if ((size_t)i + 4 > d.size()) break;
            i += 4 + (int64_t)u32((size_t)i);
        }
        return -1;
    };
    if (d.size() < 12 || std::memcmp(&d[0], "RIFF", 4) != 0 || std::memcmp(&d[8], "WAVE", 4) != 0)
        return io_fail(ARX_ERR_IO, "this doesn't seem to be a valid .WAV file");
    const int64_t di = chunk("data", 12), fi = chunk("fmt ", 12);
    if (di < 0 || fi < 0 || (size_t)fi + 24 > d.size() || (size_t)di + 8 > d.size())
        return io_fail(ARX_ERR_IO, "this doesn't seem to be a valid .WAV file");
    const size_t f = (size_t)fi;
    const uint16_t fmt = (uint16_t)u16(f + 8);
    const uint16_t nch = (uint16_t)u16(f + 10);
    const uint32_t sr = (uint32_t)u32(f + 12);
    const uint32_t bps = (uint32_t)u32(f + 16);
    const uint16_t block = (uint16_t)u16(f + 20);
    const int bits = (int)(uint16_t)u16(f + 22);
    const uint16_t bytes_per_sample = (uint16_t)(bits / 8);
    if (fmt != 1 && fmt != 3 && fmt != 0xFFFE) return io_fail(ARX_ERR_IO, "unsupported WAV encoding");
    if (nch < 1 || nch > 128) return io_fail(ARX_ERR_IO, "invalid number of channels");
    if (bps != (uint32_t)((nch * sr * (uint32_t)bits) / 8) || block != nch * bytes_per_sample)
        return io_fail(ARX_ERR_IO, "the header data in this WAV file seems to be inconsistent");
    if (bits != 8 && bits != 16 && bits != 24 && bits != 32) return io_fail(ARX_ERR_IO, "unsupported bit depth");
    const int32_t data_size = u32((size_t)di + 4);
    const int64_t n = data_size / (nch * bits / 8);
    const size_t start = (size_t)di + 8;
    float* out = (float*)std::malloc(sizeof(float) * (size_t)std::max<int64_t>(1, n * nch));
    if (!out) return io_fail(ARX_ERR_OUT_OF_MEMORY, "host allocation failed");
    for (int64_t i = 0; i < n; ++i) {
        for (int c = 0; c < nch; ++c) {
            const size_t si = start + (size_t)block * (size_t)i + (size_t)c * bytes_per_sample;
            if (si + (size_t)(bits / 8) - 1 >= d.size()) {
                std::free(out);
                return io_fail(ARX_ERR_IO, "the metadata indicates more samples than there are in the file data");
            }
            float v;
            if (bits == 8) {
                v = (float)(d[si] - 128) / 128.0f;
            } else if (bits == 16) {
                v = (float)u16(si) / 32768.0f;
            } else if (bits == 24) {
                int32_t x = (d[si + 2] << 16) | (d[si + 1] << 8) | d[si];
                if (x & 0x800000) x |= ~0xFFFFFF;
                v = (float)x / 8388608.0f;
            } else {
                int32_t x = u32(si);
                if (fmt == 3) {
                    std::memcpy(&v, &x, 4);
                } else {
                    v = (float)x / (float)2147483647;
                }
            }
            out[(size_t)c * (size_t)n + (size_t)i] = v;  // channel-major like AudioFile::samples
        }
    }
    *samples = out;
    *channels = nch;
    *frames = n;
    *sample_rate = (int32_t)sr;
    if (bit_depth) *bit_depth = bits;
    return ARX_OK;
}

void arx_free(void* p) { std::free(p); }

// AudioFile<float>::saveToWaveFile (AudioFile.h:842-955): 32-bit is always IEEE float with an
// 18-byte fmt chunk; 8/16-bit clamp to [-1,1]; 24-bit scales without clamping.
arx_status arx_wav_save(const char* path, const float* samples, int32_t channels, int64_t frames,
                        int32_t sample_rate, int32_t bit_depth) {
    if (!path || (!samples && frames > 0) || channels < 1 || channels > 128 || frames < 0)
        return io_fail(ARX_ERR_INVALID_ARGUMENT, "bad WAV parameters");
    if (bit_depth != 8 && bit_depth != 16 && bit_depth != 24 && bit_depth != 32)
        return io_fail(ARX_ERR_INVALID_ARGUMENT, "unsupported bit depth");
    const int64_t data_size64 = frames * channels * (bit_depth / 8);
    if (data_size64 > 0x7fffff00LL) return io_fail(ARX_ERR_INVALID_ARGUMENT, "WAV data exceeds 2 GiB");
    const int32_t data_size = (int32_t)data_size64;
    const bool ieee = bit_depth == 32;
    const int32_t fmt_size = ieee ? 18 : 16;
    std::vector<uint8_t> f;
    f.reserve((size_t)data_size + 64);
    auto str = [&](const char* s) { f.insert(f.end(), s, s + 4); };
    auto i32 = [&](int32_t v) {
        for (int b = 0; b < 4; ++b) f.push_back((uint8_t)(((uint32_t)v >> (8 * b)) & 0xFF));
    };
    auto i16 = [&](int16_t v) {
        f.push_back((uint8_t)(v & 0xFF));
        f.push_back((uint8_t)(((uint16_t)v >> 8) & 0xFF));
    };
    str("RIFF");
    i32(4 + fmt_size + 8 + 8 + data_size);
    str("WAVE");
    str("fmt ");
    i32(fmt_size);
    i16(ieee ? 3 : 1);
    i16((int16_t)channels);
    i32(sample_rate);
    i32((int32_t)(((int64_t)channels * sample_rate * bit_depth) / 8));
    i16((int16_t)(channels * (bit_depth / 8)));
    i16((int16_t)bit_depth);
    if (ieee) i16(0);
    str("data");
    i32(data_size);
    for (int64_t i = 0; i < frames; ++i) {
        for (int c = 0; c < channels; ++c) {
            float s = samples[(size_t)c * (size_t)frames + (size_t)i];
            if (bit_depth == 8) {
                s = std::max(std::min(s, 1.0f), -1.0f);
                s = (float)(((double)s + 1.) / 2.);
                f.push_back((uint8_t)((double)s * 255.));
            } else if (bit_depth == 16) {
                s = std::max(std::min(s, 1.0f), -1.0f);
                i16((int16_t)((double)s * 32767.));
            } else if (bit_depth == 24) {
                const int32_t x = (int32_t)(s * 8388608.0f);
                f.push_back((uint8_t)(x & 0xFF));
                f.push_back((uint8_t)((x >> 8) & 0xFF));
                f.push_back((uint8_t)((x >> 16) & 0xFF));
            } else {
                int32_t x;
                std::memcpy(&x, &s, 4);
                i32(x);
            }
        }
    }
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return io_fail(ARX_ERR_IO, std::string("cannot write ") + path);
    const size_t w = std::fwrite(f.data(), 1, f.size(), fp);
    const bool ok = (std::fclose(fp) == 0) && w == f.size();
    return ok ? ARX_OK : io_fail(ARX_ERR_IO, std::string("short write to ") + path);
}

// normalizeToRangeMinusOneToOne (R/prebuild/obj_raytracer/main.cpp:628-651): f32 min-max map
// to [-1, 1]; constant input is an error (the reference throws).
arx_status arx_normalize_min_max(float* data, size_t n) {
    if (n == 0) return ARX_OK;
    if (!data) return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    // std::min_element / max_element: first minimum / maximum under operator<
    float lo = data[0], hi = data[0];
    for (size_t i = 1; i < n; ++i) {
        if (data[i] < lo) lo = data[i];
        if (hi < data[i]) hi = data[i];
    }
    if (lo == hi) return io_fail(ARX_ERR_INVALID_ARGUMENT, "Cannot normalize: all elements in the vector are the same.");
    const float range = hi - lo;
    for (size_t i = 0; i < n; ++i) data[i] = 2.0f * ((data[i] - lo) / range) - 1.0f;
    return ARX_OK;
}

// The text dumps of AudioRenderer.cpp:525-567 / :720-744: one value per line through
// std::ostream's default float formatting (%g, precision 6).
arx_status arx_write_float_lines(const char* path, const float* data, size_t n) {
    if (!path || (!data && n)) return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    FILE* fp = std::fopen(path, "w");
    if (!fp) return io_fail(ARX_ERR_IO, std::string("cannot write ") + path);
    std::vector<char> buf(1 << 20);
    std::setvbuf(fp, buf.data(), _IOFBF, buf.size());
    for (size_t i = 0; i < n; ++i) std::fprintf(fp, "%g\n", (double)data[i]);
    const bool ok = std::fclose(fp) == 0;
    return ok ? ARX_OK : io_fail(ARX_ERR_IO, std::string("write failed: ") + path);
}

}  // extern "C"

// ----------------------------------------------------------------- JSON ----
namespace {

// A JSON value with cJSON 1.7.16's observable behaviour: numbers via strtod over the
// run of [0-9+-eE.] characters, \uXXXX (incl. surrogate pairs) to UTF-8, objects keep
// insertion order and duplicate keys, lookups are case-insensitive and first-match
// (cJSON_GetObjectItem), trailing text after the root value is accepted (cJSON_Parse).
struct Json {
    enum Kind { Null, False, True, Number, String, Array, Object } kind = Null;
    double num = 0.0;
    std::string str;
    std::vector<std::pair<std::string, Json>> items;  // Array: keys empty

    const Json* get(const char* key) const {
        if (kind != Object) return nullptr;
        for (const auto& kv : items) {
            const char* a = kv.first.c_str();
            const char* b = key;
            while (*a && std::tolower((unsigned char)*a) == std::tolower((unsigned char)*b)) {
                ++a;
                ++b;
            }
            if (std::tolower((unsigned char)*a) == std::tolower((unsigned char)*b)) return &kv.second;
        }
        return nullptr;
    }
    bool is_number() const { return kind == Number; }
    bool is_bool() const { return kind == True || kind == False; }
};

struct JsonParser {
    const char* p;
    const char* end;
    int depth = 0;

    void ws() {
        while (p < end && (unsigned char)*p <= 32) ++p;
    }
    bool lit(const char* s) {
        const size_t n = std::strlen(s);
        if ((size_t)(end - p) < n || std::strncmp(p, s, n) != 0) return false;
        p += n;
        return true;
    }
    static int hex4(const char* s) {
        int v = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = s[i];
            v <<= 4;
            if (c >= '0' && c <= '9')
                v |= c - '0';
            else if (c >= 'a' && c <= 'f')
                v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F')
                v |= c - 'A' + 10;
            else
                return -1;
        }
        return v;
    }
    bool string(std::string& out) {
        if (p >= end || *p != '"') return false;
        ++p;
        out.clear();
        while (p < end && *p != '"') {
            if (*p != '\\') {
                out.push_back(*p++);
                continue;
            }
            if (end - p < 2) return false;
            const char e = p[1];
            p += 2;
            switch (e) {
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case '"': case '\\': case '/': out.push_back(e); break;
                case 'u': {
                    if (end - p < 4) return false;
                    int cp = hex4(p);
                    if (cp < 0 || (cp >= 0xDC00 && cp <= 0xDFFF)) return false;
                    p += 4;
                    if (cp >= 0xD800 && cp <= 0xDBFF) {
                        if (end - p < 6 || p[0] != '\\' || p[1] != 'u') return false;
                        const int lo = hex4(p + 2);
                        if (lo < 0xDC00 || lo > 0xDFFF) return false;
                        p += 6;
                        cp = 0x10000 + (((cp & 0x3FF) << 10) | (lo & 0x3FF));
                    }
                    if (cp < 0x80) {
                        out.push_back((char)cp);
                    } else if (cp < 0x800) {
                        out.push_back((char)(0xC0 | (cp >> 6)));
                        out.push_back((char)(0x80 | (cp & 0x3F)));
                    } else if (cp < 0x10000) {
                        out.push_back((char)(0xE0 | (cp >> 12)));
                        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                        out.push_back((char)(0x80 | (cp & 0x3F)));
                    } else {
                        out.push_back((char)(0xF0 | (cp >> 18)));
                        out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
                        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                        out.push_back((char)(0x80 | (cp & 0x3F)));
                    }
                    break;
                }
                default: return false;
            }
        }
        if (p >= end) return false;
        ++p;
        return true;
    }
    bool value(Json& v) {
        if (++depth > 1000) return false;  // CJSON_NESTING_LIMIT
        ws();
        bool ok = value_inner(v);
        --depth;
        return ok;
    }
    bool value_inner(Json& v) {
        if (p >= end) return false;
        if (lit("null")) {
            v.kind = Json::Null;
            return true;
        }
        if (lit("false")) {
            v.kind = Json::False;
            return true;
        }
        if (lit("true")) {
            v.kind = Json::True;
            return true;
        }
        if (*p == '"') {
            v.kind = Json::String;
            return string(v.str);
        }
        if (*p == '-' || (*p >= '0' && *p <= '9')) {
            std::string buf;
            const char* q = p;
            while (q < end && (std::strchr("0123456789+-eE.", *q) != nullptr) && *q) buf.push_back(*q++);
            char* stop = nullptr;
            const double d = std::strtod(buf.c_str(), &stop);
            if (stop == buf.c_str()) return false;
            v.kind = Json::Number;
            v.num = d;
            p += (stop - buf.c_str());
            return true;
        }
        if (*p == '[' || *p == '{') {
            const bool obj = (*p == '{');
            const char close = obj ? '}' : ']';
            v.kind = obj ? Json::Object : Json::Array;
            ++p;
            ws();
            if (p < end && *p == close) {
                ++p;
                return true;
            }
            for (;;) {
                std::pair<std::string, Json> kv;
                if (obj) {
                    ws();
                    if (!string(kv.first)) return false;
                    ws();
                    if (p >= end || *p != ':') return false;
                    ++p;
                }
                if (!value(kv.second)) return false;
                v.items.push_back(std::move(kv));
                ws();
                if (p < end && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < end && *p == close) {
                    ++p;
                    return true;
                }
                return false;
            }
        }
        return false;
    }
};

bool copy_str(char* dst, size_t cap, const std::string& s) {
    if (s.size() + 1 > cap) return false;
    std::memcpy(dst, s.c_str(), s.size() + 1);
    return true;
}

// glm::vec3(x->valuedouble, ...) / gdt::vec3f(...): each component converted to float.
bool vec3_from(const Json* o, float out[3]) {
    if (!o || o->kind != Json::Object) return false;
    const Json *x = o->get("x"), *y = o->get("y"), *z = o->get("z");
    if (!(x && x->is_number() && y && y->is_number() && z && z->is_number())) return false;
    out[0] = (float)x->num;
    out[1] = (float)y->num;
    out[2] = (float)z->num;
    return true;
}

}  // namespace

extern "C" {

void arx_default_app_config(arx_app_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    // Context.cpp:19-27, 64-70, 113-119
    c->initial_volume = 1.0f;
    c->ir_length_in_seconds = 2;
    c->width = 1366;
    c->height = 768;
    c->re_render_distance_threshold = 3.0f;
    c->re_render_angle_threshold = 5.0f;
    copy_str(c->scene_file_path, sizeof(c->scene_file_path), "../../assets/models/1D_U.obj");
    c->initial_receiver_pos[0] = -2.5f;
    c->initial_receiver_pos[1] = 10.0f;
    c->base_power = 100.0f;
    c->rays[0] = c->rays[1] = c->rays[2] = 100.0f;
    c->ray_max_bounces = 10;
    c->hrtf_absorption_rate = (float)0.9;
}

arx_status arx_parse_app_config(const char* text, size_t len, arx_app_config* c) {
    if (!text || !c) return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    arx_default_app_config(c);
    JsonParser jp{text, text + len};
    if (len >= 3 && std::memcmp(text, "\xEF\xBB\xBF", 3) == 0) jp.p += 3;  // UTF-8 BOM
    Json root;
    if (!jp.value(root)) return io_fail(ARX_ERR_IO, "config: JSON parse error near offset " +
                                                        std::to_string(jp.p - text));
    const Json* it;
    const Json* rp = root.get("renderer_parameters");
    if (rp && rp->kind == Json::Object) {  // Context.cpp:28-61
        if ((it = rp->get("initial_volume")) && it->is_number()) c->initial_volume = (float)it->num;
        if ((it = rp->get("ir_length_in_seconds")) && it->is_number())
            c->ir_length_in_seconds = (uint32_t)std::round(it->num);
        if ((it = rp->get("width")) && it->is_number()) c->width = (uint32_t)std::round(it->num);
        if ((it = rp->get("height")) && it->is_number()) c->height = (uint32_t)std::round(it->num);
        if ((it = rp->get("write_first_ir_to_file")) && it->is_bool())
            c->write_first_ir_to_file = it->kind == Json::True;
        if ((it = rp->get("write_first_output_to_file")) && it->is_bool())
            c->write_first_output_to_file = it->kind == Json::True;
        if ((it = rp->get("re_render_distance_threshold")) && it->is_number())
            c->re_render_distance_threshold = (float)std::round(it->num);
        if ((it = rp->get("re_render_angle_threshold")) && it->is_number())
            c->re_render_angle_threshold = (float)std::round(it->num);
    }
    const Json* sp = root.get("scene_parameters");
    if (sp && sp->kind == Json::Object) {  // Context.cpp:71-107
        if ((it = sp->get("mono")) && it->is_bool()) c->mono = it->kind == Json::True;
        const char* keys[3] = {"scene_file_path", "audio_file_path", "materials_file_path"};
        char* dsts[3] = {c->scene_file_path, c->audio_file_path, c->materials_file_path};
        for (int k = 0; k < 3; ++k) {
            if ((it = sp->get(keys[k])) && it->kind == Json::String) {
                if (!copy_str(dsts[k], ARX_PATH_MAX, it->str))
                    return io_fail(ARX_ERR_INVALID_ARGUMENT, std::string("config: ") + keys[k] + " too long");
            }
        }
        vec3_from(sp->get("initial_receiver_pos"), c->initial_receiver_pos);
        vec3_from(sp->get("initial_emitter_pos"), c->initial_emitter_pos);
    }
    const Json* pp = root.get("pathtracer_parameters");
    if (pp && pp->kind == Json::Object) {  // Context.cpp:120-162
        if ((it = pp->get("base_power")) && it->is_number()) c->base_power = (float)it->num;
        vec3_from(pp->get("rays"), c->rays);
        if ((it = pp->get("ray_energy_threshold")) && it->is_number()) c->ray_energy_threshold = (float)it->num;
        if ((it = pp->get("ray_max_bounces")) && it->is_number())
            c->ray_max_bounces = (uint32_t)std::round(it->num);
        if ((it = pp->get("hrtf_absorption_rate")) && it->is_number())
            c->hrtf_absorption_rate = (float)std::round(it->num);
        const Json* ms = pp->get("materials");
        if (ms && ms->kind == Json::Array) {
            for (const auto& kv : ms->items) {
                const Json* n = kv.second.get("name");
                const Json* a = kv.second.get("mat_absorption");
                if (!(n && n->kind == Json::String && a && a->is_number())) continue;
                if (c->n_materials >= ARX_MAX_MATERIALS)
                    return io_fail(ARX_ERR_INVALID_ARGUMENT, "config: too many materials");
                if (!copy_str(c->material_names[c->n_materials], ARX_NAME_MAX, n->str))
                    return io_fail(ARX_ERR_INVALID_ARGUMENT, "config: material name too long");
                c->material_absorption[c->n_materials] = (float)a->num;
                ++c->n_materials;
            }
        }
    }
    return ARX_OK;
}

arx_status arx_load_app_config(const char* path, arx_app_config* c) {
    if (!path || !c) return io_fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    std::string text;
    if (!read_file(path, text)) return io_fail(ARX_ERR_IO, std::string("cannot open ") + path);
    return arx_parse_app_config(text.c_str(), text.size(), c);
}

}  // extern "C"
