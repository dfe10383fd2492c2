// arx_audio_renderer.hpp -- header-only C++ shim with the reference's AudioRenderer surface
// (R/prebuild/obj_raytracer/AudioRenderer.h:16-152) over the libarx.so C ABI (arx.h).
//
// A main.cpp-style caller keeps its call sites (main.cpp:40-67, 411-436, 547-587, 653-718):
//     OptixModel* scene = new OptixModel{loadOBJ(path)};
//     AudioRenderer* r = new AudioRenderer(scene, ir_length_in_seconds, sample_rate, materials, rays);
//     r->setMonoOutput(mono); r->setBasePower(bp); r->setThresholds(thr, max_b);
//     r->setEmitterPosInOptix(glm::vec3(...));
//     placeReceiver(sphere, scene, camera_central_point, camera.globalAngle);
//     r->setSphereCenterInOptix(glm::vec3(camera...)); r->render(&ms);
//     r->full_render_cycle(&mutex, sphere, scene, camera_central_point, angle, samples, bytes, outL, outR);
//     r->convoluteAudioFile(samples, bytes, outL, outR, &conv_ms, &proc_ms);
// Vector arguments are any type with float members x, y, z (glm::vec3, gdt::vec3f, arx::Vec3).
// placeReceiver records the receiver halves and pose in the OptixModel, as the reference's does, and
// the renderer bound to that model picks them up at the next setSphereCenterInOptix -- with a device
// refit of the receiver instead of a full GAS rebuild (OptixModel.cpp:153-257, AudioRenderer.cpp:466-486).
// Differences (documented in INTEGRATION.md): errors throw arx::Error (the reference throws
// std::runtime_error / exit()s), setters take effect at the next render without a full reload(), and
// a device list shards the rays over several GPUs (the renderer always runs through libarx's group
// API: arx_group_*, RCCL).
#pragma once

#include <chrono>
#include <cstddef>
#include <mutex>
#include <type_traits>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "arx.h"
#include "arx_circular_buffer.hpp"

namespace arx {

class Error : public std::runtime_error {
  public:
    Error(arx_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    arx_status status;
};

inline void check(arx_status s) {
    if (s != ARX_OK) throw Error(s, std::string(arx_status_string(s)) + ": " + arx_last_error());
}

struct Vec3 {
    float x, y, z;
};

// struct Material (LaunchParams.h:14-18)
struct Material {
    std::string name;
    float mat_absorption;
};

// One mesh of the scene (TriangleMesh, OptixModel.h:9-19): positions + index triples + material.
struct Mesh {
    std::vector<float> vertex;    // 3 per vertex
    std::vector<int32_t> index;   // 3 per triangle
    std::string material_name;
};

// Any vector type with float members x, y, z (glm::vec3, gdt::vec3f, Vec3).
template <class V3>
using if_vec3 = std::enable_if_t<std::is_convertible<decltype(std::declval<const V3&>().x), float>::value &&
                                 std::is_convertible<decltype(std::declval<const V3&>().z), float>::value>;
template <class V3>
inline Vec3 to_vec3(const V3& v) {
    return Vec3{(float)v.x, (float)v.y, (float)v.z};
}

// HalfSphere (HalfSphere.h: one receiver half, loaded from leftHalf.obj / rightHalf.obj in its
// local frame) and Sphere (Sphere.h:6-16: the two halves).
using HalfSphere = Mesh;
struct Sphere {
    Sphere(const HalfSphere* left, const HalfSphere* right) : left_side(left), right_side(right) {}
    const HalfSphere* left_side;
    const HalfSphere* right_side;
};

// OptixModel (OptixModel.h:21-35): the scene's meshes, plus what placeReceiver last put in it -- the
// receiver halves and the camera pose they were placed at.
struct OptixModel {
    std::vector<Mesh> meshes;
    const HalfSphere* receiver[2] = {nullptr, nullptr};
    Vec3 receiver_position{0.f, 0.f, 0.f};
    float receiver_rotation = 0.f;  // degrees, Camera::globalAngle
    uint64_t placements = 0;
};

// placeReceiver(Sphere, OptixModel*, vec3f cameraPosition, float rotation) (OptixModel.cpp:153-157):
// the halves placed at the camera, rotated by -rotation about +Y.  Here it records them; the renderer
// bound to the model re-places its receiver on the device at the next setSphereCenterInOptix.
template <class V3, class = if_vec3<V3>>
inline void placeReceiver(const Sphere& sphere, OptixModel* model, const V3& camera, float rotation) {
    model->receiver[0] = sphere.left_side;
    model->receiver[1] = sphere.right_side;
    model->receiver_position = to_vec3(camera);
    model->receiver_rotation = rotation;
    ++model->placements;
}

class AudioRenderer {
  public:
    // AudioRenderer(const OptixModel*, unsigned ir_length_in_seconds, int sample_rate,
    //               std::vector<Material>, gdt::vec3f rays_per_dimension)   (AudioRenderer.h:24), on
    // device 0 (AudioRenderer.cpp:252) or a list of GPUs; bound to the model's receiver placements
    template <class V3, class = if_vec3<V3>>
    AudioRenderer(const OptixModel* model, unsigned ir_length_in_seconds, int sample_rate,
                  std::vector<Material> materials, V3 rays_per_dimension,
                  const std::vector<int32_t>& devices = std::vector<int32_t>{0}, uint64_t seed = 1)
        : AudioRenderer(model->meshes, ir_length_in_seconds, sample_rate, materials, to_vec3(rays_per_dimension),
                        devices, seed) {
        model_ = model;
    }
    // AudioRenderer(const OptixModel*, unsigned ir_length_in_seconds, int sample_rate,
    //               std::vector<Material>, gdt::vec3f rays_per_dimension)   (AudioRenderer.h:24)
    // on one GPU (the reference hard-codes device 0, AudioRenderer.cpp:252) ...
    AudioRenderer(const std::vector<Mesh>& model, unsigned ir_length_in_seconds, int sample_rate,
                  const std::vector<Material>& materials, Vec3 rays_per_dimension, int device = 0,
                  uint64_t seed = 1)
        : AudioRenderer(model, ir_length_in_seconds, sample_rate, materials, rays_per_dimension,
                        std::vector<int32_t>{(int32_t)device}, seed) {}
    // ... or ray-sharded over several GPUs of this process (arx_group_create: RCCL all-reduce of
    // the IR histogram; render() returns once every GPU holds the full IR).
    AudioRenderer(const std::vector<Mesh>& model, unsigned ir_length_in_seconds, int sample_rate,
                  const std::vector<Material>& materials, Vec3 rays_per_dimension, const std::vector<int32_t>& devices,
                  uint64_t seed = 1) {
        arx_config c;
        arx_default_config(&c);
        c.rays_x = (int32_t)rays_per_dimension.x;
        c.rays_y = (int32_t)rays_per_dimension.y;
        c.rays_z = (int32_t)rays_per_dimension.z;
        c.ir_length_in_seconds = ir_length_in_seconds;
        c.sample_rate = sample_rate;
        c.seed = seed;
        check(arx_group_create(&c, devices.data(), (int32_t)devices.size(), &g_));
        h_ = arx_group_member(g_, 0);
        ir_length_ = (size_t)ir_length_in_seconds * (size_t)sample_rate;
        setScene(model, materials);
    }
    ~AudioRenderer() { arx_group_destroy(g_); }
    AudioRenderer(const AudioRenderer&) = delete;
    AudioRenderer& operator=(const AudioRenderer&) = delete;

    // buildAccel + buildSBT with getMaterialAbsorption (AudioRenderer.cpp:34-56, 95-218, 413-464)
    void setScene(const std::vector<Mesh>& model, const std::vector<Material>& materials) {
        std::vector<const char*> names;
        std::vector<float> abs;
        for (const auto& m : materials) {
            names.push_back(m.name.c_str());
            abs.push_back(m.mat_absorption);
        }
        std::vector<float> tv, ta;
        for (const auto& mesh : model) {
            const float a = arx_material_absorption(mesh.material_name.c_str(), names.data(), abs.data(), names.size());
            for (size_t t = 0; t + 2 < mesh.index.size(); t += 3) {
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < 3; ++c) tv.push_back(mesh.vertex[3 * (size_t)mesh.index[t + k] + c]);
                ta.push_back(a);
            }
        }
        check(arx_group_set_scene(g_, tv.data(), ta.data(), (int64_t)ta.size()));
    }
    // HalfSphere meshes (leftHalf.obj / rightHalf.obj) in their local frame.
    void setReceiverModel(const Mesh& left, const Mesh& right) {
        const Mesh* m[2] = {&left, &right};
        for (int side = 0; side < 2; ++side) {
            std::vector<float> tv;
            for (size_t t = 0; t + 2 < m[side]->index.size(); t += 3)
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < 3; ++c) tv.push_back(m[side]->vertex[3 * (size_t)m[side]->index[t + k] + c]);
            check(arx_group_set_receiver_model(g_, side, tv.data(), (int64_t)(tv.size() / 9)));
        }
    }

    // :27 -- with the write-IR flag set, the IR is dumped once to output_ir_{left,right}.txt
    // (experimentation/output_ir_*_<stamp>.txt in experimentation mode) and the flag cleared, as
    // AudioRenderer.cpp:525-567 does
    void render(double* render_time = nullptr) {
        check(arx_group_render(g_, render_time));
        if (!render_time) check(arx_group_synchronize(g_));
        if (!write_ir_) return;
        std::vector<float> l(ir_length_), r(ir_length_);
        getIR(l.data(), r.data());
        std::string lp = "output_ir_left.txt", rp = "output_ir_right.txt";
        if (experimentation_) {
            const std::string stamp = std::to_string(std::chrono::system_clock::now().time_since_epoch().count());
            lp = "experimentation/output_ir_left_" + stamp + ".txt";
            rp = "experimentation/output_ir_right_" + stamp + ".txt";
        }
        check(arx_write_float_lines(lp.c_str(), l.data(), l.size()));
        check(arx_write_float_lines(rp.c_str(), r.data(), r.size()));
        write_ir_ = false;
    }

    // :31 -- sizes in bytes, host buffers owned by the caller (on several GPUs, each convolves its
    // time-block shard: arx_group_convolute_audio_file, bit-identical to one GPU); with the
    // write-output flag set, the result is dumped once to output_convolute_{left,right}.txt and the
    // flag cleared (AudioRenderer.cpp:720-744)
    void convoluteAudioFile(float* h_inputBuffer, size_t h_inputBufferSize, float* h_outputBuffer_left,
                            float* h_outputBuffer_right, double* convolute_time = nullptr,
                            double* convolute_process_time = nullptr) {
        check(arx_group_convolute_audio_file(g_, h_inputBuffer, h_inputBufferSize, h_outputBuffer_left,
                                             h_outputBuffer_right, convolute_time, convolute_process_time));
        if (!write_output_) return;
        const size_t n = h_inputBufferSize / sizeof(float);
        check(arx_write_float_lines("output_convolute_left.txt", h_outputBuffer_left, n));
        check(arx_write_float_lines("output_convolute_right.txt", h_outputBuffer_right, n));
        write_output_ = false;
    }

    void setEmitterPosInOptix(Vec3 p) { check(arx_group_set_emitter(g_, p.x, p.y, p.z)); }  // :33
    template <class V3, class = if_vec3<V3>>
    void setEmitterPosInOptix(const V3& p) {  // setEmitterPosInOptix(glm::vec3) (AudioRenderer.h:33)
        setEmitterPosInOptix(to_vec3(p));
    }
    // placeReceiver(sphere, model, camera, yaw) + setSphereCenterInOptix(camera) in one call
    void setSphereCenterInOptix(Vec3 p, float yaw_deg) { check(arx_group_set_listener(g_, p.x, p.y, p.z, yaw_deg)); }
    // setSphereCenterInOptix(glm::vec3) (AudioRenderer.h:35): the listener at p; on a renderer bound to
    // an OptixModel, the receiver halves and rotation of the model's last placeReceiver (a new pair of
    // halves is uploaded once), else the receiver model set by setReceiverModel at yaw 0
    void setSphereCenterInOptix(Vec3 p) {
        float yaw = 0.0f;
        if (model_ && model_->placements) {
            if (model_->receiver[0] && model_->receiver[1] &&
                (model_->receiver[0] != bound_[0] || model_->receiver[1] != bound_[1])) {
                setReceiverModel(*model_->receiver[0], *model_->receiver[1]);
                bound_[0] = model_->receiver[0];
                bound_[1] = model_->receiver[1];
            }
            yaw = model_->receiver_rotation;
        }
        setSphereCenterInOptix(p, yaw);
    }
    template <class V3, class = if_vec3<V3>>
    void setSphereCenterInOptix(const V3& p) {
        setSphereCenterInOptix(to_vec3(p));
    }
    void setThresholds(float energy, unsigned int max_bounces) { check(arx_group_set_thresholds(g_, energy, max_bounces)); }
    void set_hrtf_absorption_rate(float v) { check(arx_group_set_hrtf_absorption_rate(g_, v)); }
    void setBasePower(float v) { check(arx_group_set_base_power(g_, v)); }
    void setMonoOutput(bool v) { check(arx_group_set_mono_output(g_, v ? 1 : 0)); }
    // Not in the reference: 2 lets a render / convolute loop keep two frames in flight
    // (arx_set_frames_in_flight; results bit-identical to one frame at a time)
    void setFramesInFlight(int n) { check(arx_group_set_frames_in_flight(g_, n)); }
    // :47 -- declared by the reference, body empty (AudioRenderer.cpp:574-576); kept for source
    // compatibility, it does nothing (the live path zips L/R in pass_d_live)
    void normalizeAndMergeStereoOutput(double*, double*, size_t, double*) {}

    // full_render_cycle(std::mutex*, Sphere, OptixModel*, gdt::vec3f, float, float*, size_t, float*,
    // float*) (AudioRenderer.h:49, AudioRenderer.cpp:790-798): under the caller's mutex, place the
    // receiver at the camera, move the listener there, render, convolve the file
    template <class V3, class = if_vec3<V3>>
    void full_render_cycle(std::mutex* mutex, const Sphere& sphere, OptixModel* scene, const V3& camera_central_point,
                           float camera_global_angle, float* audio_samples, size_t size_of_audio,
                           float* outputBuffer_left, float* outputBuffer_right) {
        std::lock_guard<std::mutex> lock(*mutex);
        if (scene && scene == model_) {
            placeReceiver(sphere, scene, camera_central_point, camera_global_angle);
            setSphereCenterInOptix(to_vec3(camera_central_point));
        } else {  // a renderer not bound to this model: the halves and pose straight from the arguments
            if (sphere.left_side && sphere.right_side) setReceiverModel(*sphere.left_side, *sphere.right_side);
            setSphereCenterInOptix(to_vec3(camera_central_point), camera_global_angle);
        }
        render();
        convoluteAudioFile(audio_samples, size_of_audio, outputBuffer_left, outputBuffer_right);
    }
    // the same without the mutex and the Sphere (callers that keep their own lock)
    void full_render_cycle(Vec3 camera, float yaw_deg, float* audio, size_t bytes, float* outL, float* outR) {
        setSphereCenterInOptix(camera, yaw_deg);
        render();
        convoluteAudioFile(audio, bytes, outL, outR);
    }

    // :29 -- one mic block (f64, bytes) convolved with both IRs; 2*ir_len zipped L/R values are
    // added into the caller's CircularBuffer (AudioRenderer.cpp:593-661)
    void convoluteLiveInput(double* h_inputBuffer, size_t h_inputBufferSize, CircularBuffer<double>* samplesRecordBuffer) {
        live_scratch_.resize(2 * ir_length_);
        check(arx_convolute_live_block(h_, h_inputBuffer, h_inputBufferSize, live_scratch_.data(), live_scratch_.size()));
        if (samplesRecordBuffer) samplesRecordBuffer->add(live_scratch_.data(), live_scratch_.size());
    }

    // text dumps (AudioRenderer.cpp:525-567, 720-744; setters :780-788): the next render() writes
    // output_ir_{left,right}.txt, the next convoluteAudioFile() output_convolute_{left,right}.txt
    void set_write_ir_to_file_flag(bool v) { write_ir_ = v; }
    void set_write_output_to_file_flag(bool v) { write_output_ = v; }
    void enable_experimentation() { experimentation_ = true; }

    void getIR(float* left, float* right) { check(arx_group_copy_ir(g_, left, right, ir_length_)); }
    arx_stats stats() {
        arx_stats s;
        check(arx_group_get_stats(g_, &s));
        return s;
    }
    size_t irLength() const { return ir_length_; }
    int gpuCount() const { return arx_group_ranks(g_); }
    arx_renderer* handle() { return h_; }  // the first GPU's renderer
    arx_group* group() { return g_; }

  private:
    arx_group* g_ = nullptr;
    arx_renderer* h_ = nullptr;  // member 0, owned by g_
    const OptixModel* model_ = nullptr;        // the model whose receiver placements this renderer follows
    const HalfSphere* bound_[2] = {nullptr, nullptr};  // the halves uploaded last
    size_t ir_length_ = 0;
    std::vector<double> live_scratch_;
    bool write_ir_ = false, write_output_ = false, experimentation_ = false;
};

// ---- input / output formats over libarx.so's native readers ------------------------------

// loadOBJ (OptixModel.cpp:75-151): one Mesh per (shape, material), names = material names.
inline std::vector<Mesh> loadOBJ(const std::string& path) {
    arx_model* m = nullptr;
    check(arx_model_load_obj(path.c_str(), nullptr, 0, nullptr, &m));
    std::vector<Mesh> out;
    for (int64_t i = 0; i < arx_model_mesh_count(m); ++i) {
        const char* name = nullptr;
        const float* v = nullptr;
        const int32_t* idx = nullptr;
        int64_t nv = 0, nt = 0;
        const arx_status st = arx_model_mesh(m, i, &name, &v, &nv, &idx, &nt);
        if (st != ARX_OK) {
            arx_model_free(m);
            check(st);
        }
        Mesh mesh;
        mesh.material_name = name ? name : "";
        mesh.vertex.assign(v, v + 3 * nv);
        mesh.index.assign(idx, idx + 3 * nt);
        out.push_back(std::move(mesh));
    }
    arx_model_free(m);
    return out;
}

// HalfSphere(objFile) + place_receiver_half's mesh of shapes[0] (HalfSphere.cpp:3-31,
// OptixModel.cpp:197-220), local frame; the last material mesh wins like the reference.
inline Mesh loadHalfSphere(const std::string& path, bool left) {
    arx_model* m = nullptr;
    const std::string dir = path.substr(0, path.rfind('/'));
    check(arx_model_load_obj(path.c_str(), dir.c_str(), 1, left ? "receiver_left" : "receiver_right", &m));
    Mesh mesh;
    const int64_t n = arx_model_mesh_count(m);
    if (n > 0) {
        const char* name = nullptr;
        const float* v = nullptr;
        const int32_t* idx = nullptr;
        int64_t nv = 0, nt = 0;
        arx_model_mesh(m, n - 1, &name, &v, &nv, &idx, &nt);
        mesh.material_name = name;
        mesh.vertex.assign(v, v + 3 * nv);
        mesh.index.assign(idx, idx + 3 * nt);
    }
    arx_model_free(m);
    return mesh;
}

// AudioFile<float> load / save (AudioFile.h): samples[channel][frame]
struct Wav {
    std::vector<std::vector<float>> samples;
    int32_t sample_rate = 44100;
    int32_t bit_depth = 16;
};

inline Wav loadWav(const std::string& path) {
    float* data = nullptr;
    int32_t ch = 0, sr = 0, bits = 0;
    int64_t n = 0;
    check(arx_wav_load(path.c_str(), &data, &ch, &n, &sr, &bits));
    Wav w;
    w.sample_rate = sr;
    w.bit_depth = bits;
    for (int32_t c = 0; c < ch; ++c) w.samples.emplace_back(data + (size_t)c * n, data + (size_t)(c + 1) * n);
    arx_free(data);
    return w;
}

inline void saveWav(const std::string& path, const Wav& w) {
    const size_t n = w.samples.empty() ? 0 : w.samples[0].size();
    std::vector<float> flat;
    for (const auto& c : w.samples) flat.insert(flat.end(), c.begin(), c.end());
    check(arx_wav_save(path.c_str(), flat.data(), (int32_t)w.samples.size(), (int64_t)n, w.sample_rate, w.bit_depth));
}

// normalizeToRangeMinusOneToOne (main.cpp:628-651)
inline std::vector<float> normalizeToRangeMinusOneToOne(std::vector<float> v) {
    check(arx_normalize_min_max(v.data(), v.size()));
    return v;
}

// Context::loadContext's parameters (Context.cpp:15-164); materials as the renderer takes them
inline arx_app_config loadConfig(const std::string& path) {
    arx_app_config c;
    check(arx_load_app_config(path.c_str(), &c));
    return c;
}

inline std::vector<Material> configMaterials(const arx_app_config& c) {
    std::vector<Material> m;
    for (int32_t i = 0; i < c.n_materials; ++i) m.push_back({c.material_names[i], c.material_absorption[i]});
    return m;
}

}  // namespace arx
