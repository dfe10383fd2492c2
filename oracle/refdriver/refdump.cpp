// refdump -- fixture generator driver (TEST INFRASTRUCTURE, built by `make -C oracle ref`).
//
// Links the reference's own input-side code, compiled from /root/reference where it
// lies (never copied): tinyobj v2.0.0 (prebuild/common/3rdParty/tiny_obj_loader.h),
// AudioFile.h and cJSON.c (prebuild/obj_raytracer/), glm 0.9.9 (prebuild/common/glm).
// OptixModel.cpp / Context.cpp themselves need OptiX headers, so the few lines of
// glue they add on top of those libraries (per-material split with vertex dedup,
// receiver transform, config defaults) are restated here with file:line cites.
// Output goes to stdout; tests/golden/make_golden.py turns it into fixtures.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"
#include "AudioFile.h"
extern "C" {
#include "cJSON.h"
}
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>

#include <cmath>
#include <cstdio>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Key {
    int v, n, t;
    bool operator<(const Key& o) const {  // OptixModel.cpp:13-32 ordering
        if (v != o.v) return v < o.v;
        if (n != o.n) return n < o.n;
        return t < o.t;
    }
};

struct MeshOut {
    std::string name;
    std::vector<float> v;
    std::vector<int> idx;
};

// OptixModel.cpp:37-72 addVertex (positions only matter downstream)
int add_vertex(MeshOut& m, const std::vector<float>& verts, const tinyobj::index_t& i,
               std::map<Key, int>& known) {
    Key k{i.vertex_index, i.normal_index, i.texcoord_index};
    auto it = known.find(k);
    if (it != known.end()) return it->second;
    int id = (int)(m.v.size() / 3);
    known[k] = id;
    for (int c = 0; c < 3; ++c) m.v.push_back(verts[3 * i.vertex_index + c]);
    return id;
}

// OptixModel.cpp:104-141: one mesh per (shape, material id in ascending order)
void split_shapes(const std::vector<tinyobj::shape_t>& shapes, const std::vector<float>& verts,
                  const std::vector<tinyobj::material_t>& mats, const char* forced_name,
                  std::vector<MeshOut>& out) {
    for (const auto& shape : shapes) {
        std::set<int> ids(shape.mesh.material_ids.begin(), shape.mesh.material_ids.end());
        for (int mid : ids) {
            MeshOut m;
            std::map<Key, int> known;
            for (size_t f = 0; f < shape.mesh.material_ids.size(); ++f) {
                if (shape.mesh.material_ids[f] != mid) continue;
                for (int c = 0; c < 3; ++c)
                    m.idx.push_back(add_vertex(m, verts, shape.mesh.indices[3 * f + c], known));
                if (forced_name)
                    m.name = forced_name;
                else if (mid >= 0)
                    m.name = mats[mid].name;
            }
            if (!m.v.empty()) out.push_back(m);
        }
        if (forced_name) break;  // place_receiver_half uses side.shapes[0] only (OptixModel.cpp:197-220)
    }
}

void dump_meshes(const std::vector<MeshOut>& ms) {
    std::printf("meshes %zu\n", ms.size());
    for (const auto& m : ms) {
        std::printf("mesh %s %zu %zu\n", m.name.empty() ? "<none>" : m.name.c_str(), m.v.size() / 3,
                    m.idx.size() / 3);
        for (size_t i = 0; i < m.v.size(); ++i) std::printf("%a\n", m.v[i]);
        for (size_t i = 0; i < m.idx.size(); ++i) std::printf("%d\n", m.idx[i]);
    }
}

bool load(const std::string& path, const std::string& mtl_dir, tinyobj::attrib_t& a,
          std::vector<tinyobj::shape_t>& s, std::vector<tinyobj::material_t>& m) {
    std::string err;
    return tinyobj::LoadObj(&a, &s, &m, &err, &err, path.c_str(), mtl_dir.c_str(), true);
}

int cmd_obj(const std::string& path) {
    tinyobj::attrib_t a;
    std::vector<tinyobj::shape_t> s;
    std::vector<tinyobj::material_t> m;
    // OptixModel.cpp:79: mtlDir = objFile.substr(0, objFile.rfind('/') + 1)
    if (!load(path, path.substr(0, path.rfind('/') + 1), a, s, m)) return 2;
    std::printf("shapes %zu materials %zu vertices %zu\n", s.size(), m.size(), a.vertices.size() / 3);
    std::vector<MeshOut> out;
    split_shapes(s, a.vertices, m, nullptr, out);
    dump_meshes(out);
    return 0;
}

// OptixModel.cpp:159-257 place_receiver_half, left then right (placeReceiver :153-157)
int cmd_receiver(const std::string& left, const std::string& right, float x, float y, float z,
                 float yaw) {
    std::vector<MeshOut> out;
    const char* names[2] = {"receiver_left", "receiver_right"};
    const std::string paths[2] = {left, right};
    for (int side = 0; side < 2; ++side) {
        tinyobj::attrib_t a;
        std::vector<tinyobj::shape_t> s;
        std::vector<tinyobj::material_t> m;
        // HalfSphere.cpp:5: mtlDir = objFile.substr(0, objFile.rfind('/'))
        if (!load(paths[side], paths[side].substr(0, paths[side].rfind('/')), a, s, m)) return 2;
        std::vector<float> moved = a.vertices;
        std::set<int> uniq;
        for (const auto& sh : s)
            for (const auto& i : sh.mesh.indices) uniq.insert(i.vertex_index);
        for (int index : uniq) {
            float ang = glm::radians(yaw);
            glm::mat4 R = glm::rotate(glm::mat4(1.0f), -ang, glm::vec3(0, 1, 0));
            glm::vec4 v = glm::vec4(a.vertices[3 * index + 0], a.vertices[3 * index + 1],
                                    a.vertices[3 * index + 2], 1.0);
            v = R * v;
            moved[3 * index + 0] = x + v.x;
            moved[3 * index + 1] = y + v.y;
            moved[3 * index + 2] = z + v.z;
        }
        split_shapes(s, moved, m, names[side], out);
    }
    dump_meshes(out);
    return 0;
}

int cmd_wav(const std::string& path) {
    AudioFile<float> f;
    if (!f.load(path)) return 2;
    std::printf("wav %u %d %d %d\n", f.getSampleRate(), f.getNumChannels(), f.getNumSamplesPerChannel(),
                f.getBitDepth());
    for (int c = 0; c < f.getNumChannels(); ++c)
        for (float v : f.samples[c]) std::printf("%a\n", v);
    return 0;
}

// Context.cpp:15-164 (defaults + rounding quirks)
int cmd_config(const std::string& path) {
    std::ifstream in(path);
    std::stringstream ss;
    ss << in.rdbuf();
    cJSON* cfg = cJSON_Parse(ss.str().c_str());
    if (!cfg) return 2;
    double initial_volume = 1.0, ir_sec = 2, width = 1366, height = 768, rr_dist = 3, rr_ang = 5;
    int wir = 0, wout = 0, mono = 0;
    std::string scene = "../../assets/models/1D_U.obj", audio, mats_path;
    float rx = -2.5f, ry = 10.0f, rz = 0.0f, ex = 0, ey = 0, ez = 0;
    float base_power = 100.f, thr = 0.f, hrtf = 0.9f;
    double rays[3] = {100, 100, 100};
    unsigned max_b = 10;
    std::vector<std::pair<std::string, float>> mats;
    const cJSON* r = cJSON_GetObjectItem(cfg, "renderer_parameters");
    if (cJSON_IsObject(r)) {
        const cJSON* it;
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "initial_volume"))) initial_volume = (float)it->valuedouble;
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "ir_length_in_seconds"))) ir_sec = (unsigned)std::round(it->valuedouble);
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "width"))) width = (unsigned)std::round(it->valuedouble);
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "height"))) height = (unsigned)std::round(it->valuedouble);
        if (cJSON_IsBool(it = cJSON_GetObjectItem(r, "write_first_ir_to_file"))) wir = cJSON_IsTrue(it);
        if (cJSON_IsBool(it = cJSON_GetObjectItem(r, "write_first_output_to_file"))) wout = cJSON_IsTrue(it);
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "re_render_distance_threshold"))) rr_dist = (float)std::round(it->valuedouble);
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(r, "re_render_angle_threshold"))) rr_ang = (float)std::round(it->valuedouble);
    }
    const cJSON* sp = cJSON_GetObjectItem(cfg, "scene_parameters");
    if (cJSON_IsObject(sp)) {
        const cJSON* it;
        if (cJSON_IsBool(it = cJSON_GetObjectItem(sp, "mono"))) mono = cJSON_IsTrue(it);
        if (cJSON_IsString(it = cJSON_GetObjectItem(sp, "scene_file_path"))) scene = it->valuestring;
        if (cJSON_IsString(it = cJSON_GetObjectItem(sp, "audio_file_path"))) audio = it->valuestring;
        if (cJSON_IsString(it = cJSON_GetObjectItem(sp, "materials_file_path"))) mats_path = it->valuestring;
        const cJSON* p = cJSON_GetObjectItem(sp, "initial_receiver_pos");
        if (cJSON_IsObject(p)) {
            cJSON *x = cJSON_GetObjectItem(p, "x"), *y = cJSON_GetObjectItem(p, "y"), *z = cJSON_GetObjectItem(p, "z");
            if (cJSON_IsNumber(x) && cJSON_IsNumber(y) && cJSON_IsNumber(z)) {
                rx = (float)x->valuedouble; ry = (float)y->valuedouble; rz = (float)z->valuedouble;
            }
        }
        p = cJSON_GetObjectItem(sp, "initial_emitter_pos");
        if (cJSON_IsObject(p)) {
            cJSON *x = cJSON_GetObjectItem(p, "x"), *y = cJSON_GetObjectItem(p, "y"), *z = cJSON_GetObjectItem(p, "z");
            if (cJSON_IsNumber(x) && cJSON_IsNumber(y) && cJSON_IsNumber(z)) {
                ex = (float)x->valuedouble; ey = (float)y->valuedouble; ez = (float)z->valuedouble;
            }
        }
    }
    const cJSON* pp = cJSON_GetObjectItem(cfg, "pathtracer_parameters");
    if (cJSON_IsObject(pp)) {
        const cJSON* it;
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(pp, "base_power"))) base_power = (float)it->valuedouble;
        const cJSON* rs = cJSON_GetObjectItem(pp, "rays");
        if (cJSON_IsObject(rs)) {
            cJSON *x = cJSON_GetObjectItem(rs, "x"), *y = cJSON_GetObjectItem(rs, "y"), *z = cJSON_GetObjectItem(rs, "z");
            if (cJSON_IsNumber(x) && cJSON_IsNumber(y) && cJSON_IsNumber(z)) {
                rays[0] = (float)x->valuedouble; rays[1] = (float)y->valuedouble; rays[2] = (float)z->valuedouble;
            }
        }
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(pp, "ray_energy_threshold"))) thr = (float)it->valuedouble;
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(pp, "ray_max_bounces"))) max_b = (unsigned)std::round(it->valuedouble);
        if (cJSON_IsNumber(it = cJSON_GetObjectItem(pp, "hrtf_absorption_rate"))) hrtf = (float)std::round(it->valuedouble);
        const cJSON* ms = cJSON_GetObjectItem(pp, "materials");
        const cJSON* m = nullptr;
        if (cJSON_IsArray(ms)) {
            cJSON_ArrayForEach(m, ms) {
                cJSON* n = cJSON_GetObjectItem(m, "name");
                cJSON* ab = cJSON_GetObjectItem(m, "mat_absorption");
                if (cJSON_IsString(n) && cJSON_IsNumber(ab)) mats.push_back({n->valuestring, (float)ab->valuedouble});
            }
        }
    }
    std::printf("initial_volume %a\nir_length_in_seconds %u\nwidth %u\nheight %u\n", (float)initial_volume,
                (unsigned)ir_sec, (unsigned)width, (unsigned)height);
    std::printf("write_first_ir_to_file %d\nwrite_first_output_to_file %d\n", wir, wout);
    std::printf("re_render_distance_threshold %a\nre_render_angle_threshold %a\n", (float)rr_dist, (float)rr_ang);
    std::printf("mono %d\nscene_file_path %s\naudio_file_path %s\nmaterials_file_path %s\n", mono, scene.c_str(),
                audio.empty() ? "<none>" : audio.c_str(), mats_path.empty() ? "<none>" : mats_path.c_str());
    std::printf("initial_receiver_pos %a %a %a\ninitial_emitter_pos %a %a %a\n", rx, ry, rz, ex, ey, ez);
    std::printf("base_power %a\nrays %a %a %a\nray_energy_threshold %a\nray_max_bounces %u\nhrtf_absorption_rate %a\n",
                base_power, (float)rays[0], (float)rays[1], (float)rays[2], thr, max_b, hrtf);
    for (auto& m : mats) std::printf("material %s %a\n", m.first.c_str(), m.second);
    cJSON_Delete(cfg);
    return 0;
}

std::vector<float> read_raw(const std::string& path, size_t n) {
    std::vector<float> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f || std::fread(v.data(), sizeof(float), n, f) != n) v.clear();
    if (f) std::fclose(f);
    return v;
}

// AudioFile<float>::save of a channel-major raw f32 buffer (export_audio, main.cpp:709-716)
int cmd_wavsave(const std::string& raw, int ch, int n, int sr, int bits, const std::string& out) {
    std::vector<float> v = read_raw(raw, (size_t)ch * n);
    if (v.empty() && ch * n) return 2;
    std::vector<std::vector<float>> buf(ch, std::vector<float>(n));
    for (int c = 0; c < ch; ++c)
        for (int i = 0; i < n; ++i) buf[c][i] = v[(size_t)c * n + i];
    AudioFile<float> f;
    f.setAudioBuffer(buf);
    f.setSampleRate(sr);
    f.setBitDepth(bits);
    return f.save(out) ? 0 : 3;
}

// the IR / output text dumps: std::ofstream << float << std::endl (AudioRenderer.cpp:552-556)
int cmd_lines(const std::string& raw, int n, const std::string& out) {
    std::vector<float> v = read_raw(raw, (size_t)n);
    std::ofstream o(out);
    for (int i = 0; i < n; ++i) o << v[i] << std::endl;
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: refdump obj|receiver|wav|config ...\n");
        return 1;
    }
    std::string cmd = argv[1];
    if (cmd == "obj") return cmd_obj(argv[2]);
    if (cmd == "wav") return cmd_wav(argv[2]);
    if (cmd == "config") return cmd_config(argv[2]);
    if (cmd == "wavsave" && argc >= 8)
        return cmd_wavsave(argv[2], std::stoi(argv[3]), std::stoi(argv[4]), std::stoi(argv[5]), std::stoi(argv[6]),
                           argv[7]);
    if (cmd == "lines" && argc >= 5) return cmd_lines(argv[2], std::stoi(argv[3]), argv[4]);
    if (cmd == "receiver" && argc >= 8)
        return cmd_receiver(argv[2], argv[3], std::stof(argv[4]), std::stof(argv[5]), std::stof(argv[6]),
                            std::stof(argv[7]));
    return 1;
}
