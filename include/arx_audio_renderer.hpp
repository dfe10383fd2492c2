// arx_audio_renderer.hpp -- header-only C++ shim with the reference's AudioRenderer surface
// (R/prebuild/obj_raytracer/AudioRenderer.h:16-152) over the libarx.so C ABI (arx.h).
//
// A main.cpp-style caller keeps its call sites:
//     AudioRenderer* r = new AudioRenderer(scene_tris, ir_length_in_seconds, sample_rate, materials, rays);
//     r->setMonoOutput(mono); r->setBasePower(bp); r->setThresholds(thr, max_b);
//     r->setEmitterPosInOptix(emitter); r->setSphereCenterInOptix(camera_pos);
//     r->render(&ms); r->convoluteAudioFile(samples, bytes, outL, outR, &conv_ms, &proc_ms);
// Differences (documented in INTEGRATION.md): the scene is passed as flat triangles with
// material names instead of an OptixModel*, errors throw arx::Error (the reference
// throws std::runtime_error / exit()s), and setters take effect at the next render
// without a full reload().
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "arx.h"

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

class AudioRenderer {
  public:
    // AudioRenderer(const OptixModel*, unsigned ir_length_in_seconds, int sample_rate,
    //               std::vector<Material>, gdt::vec3f rays_per_dimension)   (AudioRenderer.h:24)
    AudioRenderer(const std::vector<Mesh>& model, unsigned ir_length_in_seconds, int sample_rate,
                  const std::vector<Material>& materials, Vec3 rays_per_dimension, int device = 0,
                  uint64_t seed = 1) {
        arx_config c;
        arx_default_config(&c);
        c.rays_x = (int32_t)rays_per_dimension.x;
        c.rays_y = (int32_t)rays_per_dimension.y;
        c.rays_z = (int32_t)rays_per_dimension.z;
        c.ir_length_in_seconds = ir_length_in_seconds;
        c.sample_rate = sample_rate;
        c.device = device;
        c.seed = seed;
        check(arx_create(&c, &h_));
        ir_length_ = (size_t)ir_length_in_seconds * (size_t)sample_rate;
        setScene(model, materials);
    }
    ~AudioRenderer() { arx_destroy(h_); }
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
        check(arx_set_scene(h_, tv.data(), ta.data(), (int64_t)ta.size()));
    }
    // HalfSphere meshes (leftHalf.obj / rightHalf.obj) in their local frame.
    void setReceiverModel(const Mesh& left, const Mesh& right) {
        const Mesh* m[2] = {&left, &right};
        for (int side = 0; side < 2; ++side) {
            std::vector<float> tv;
            for (size_t t = 0; t + 2 < m[side]->index.size(); t += 3)
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < 3; ++c) tv.push_back(m[side]->vertex[3 * (size_t)m[side]->index[t + k] + c]);
            check(arx_set_receiver_model(h_, side, tv.data(), (int64_t)(tv.size() / 9)));
        }
    }

    void render(double* render_time = nullptr) { check(arx_render(h_, render_time)); }  // :27

    // :31 -- sizes in bytes, host buffers owned by the caller
    void convoluteAudioFile(float* h_inputBuffer, size_t h_inputBufferSize, float* h_outputBuffer_left,
                            float* h_outputBuffer_right, double* convolute_time = nullptr,
                            double* convolute_process_time = nullptr) {
        check(arx_convolute_audio_file(h_, h_inputBuffer, h_inputBufferSize, h_outputBuffer_left, h_outputBuffer_right,
                                       convolute_time, convolute_process_time));
    }

    void setEmitterPosInOptix(Vec3 p) { check(arx_set_emitter(h_, p.x, p.y, p.z)); }          // :33
    // placeReceiver(sphere, model, camera, yaw) + setSphereCenterInOptix(camera) in one call
    void setSphereCenterInOptix(Vec3 p, float yaw_deg = 0.0f) { check(arx_set_listener(h_, p.x, p.y, p.z, yaw_deg)); }
    void setThresholds(float energy, unsigned int max_bounces) { check(arx_set_thresholds(h_, energy, max_bounces)); }
    void set_hrtf_absorption_rate(float v) { check(arx_set_hrtf_absorption_rate(h_, v)); }
    void setBasePower(float v) { check(arx_set_base_power(h_, v)); }
    void setMonoOutput(bool v) { check(arx_set_mono_output(h_, v ? 1 : 0)); }

    // full_render_cycle (AudioRenderer.cpp:790-798) minus the mutex (callers keep theirs)
    void full_render_cycle(Vec3 camera, float yaw_deg, float* audio, size_t bytes, float* outL, float* outR) {
        setSphereCenterInOptix(camera, yaw_deg);
        render();
        convoluteAudioFile(audio, bytes, outL, outR);
    }

    void getIR(float* left, float* right) { check(arx_copy_ir(h_, left, right, ir_length_)); }
    arx_stats stats() {
        arx_stats s;
        check(arx_get_stats(h_, &s));
        return s;
    }
    size_t irLength() const { return ir_length_; }
    arx_renderer* handle() { return h_; }

  private:
    arx_renderer* h_ = nullptr;
    size_t ir_length_ = 0;
};

}  // namespace arx
