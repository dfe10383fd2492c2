// main_style_demo -- the reference's full_render (R/prebuild/obj_raytracer/main.cpp:40-67) against the
// C++ shim (include/arx_audio_renderer.hpp), with the reference's own call sites: an OptixModel*, a
// Sphere of two HalfSpheres, a gdt::vec3f camera point, glm::vec3 setters, placeReceiver and
// full_render_cycle(std::mutex*, Sphere, OptixModel*, vec3f, float, ...).
//
//   main_style_demo config.json leftHalf.obj rightHalf.obj out_dir angle_deg
//
// File branch (isLive = false) at the config's receiver position and camera angle angle_deg, then the
// live branch (isLive = true) with the camera moved by (+0.5, 0, -0.25) and turned by 30 deg.  Writes
// ir_file_{left,right}.f32, conv_{left,right}.f32, ir_live_{left,right}.f32 to out_dir.
//
// Built with -DARX_DEMO_GLM and the reference's glm on the include path, glm::vec3 is glm's own
// (tests/test_shim_host.py, compile only); otherwise a stand-in with the members the call sites use.
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "arx_audio_renderer.hpp"

#ifdef ARX_DEMO_GLM
#include <glm/glm.hpp>
#else
namespace glm {
struct vec3 {
    float x, y, z;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};
}  // namespace glm
#endif
namespace gdt {  // gdt/math/vec.h's vec3f: the reference's launch-side vector type
struct vec3f {
    float x, y, z;
    vec3f(float a, float b, float c) : x(a), y(b), z(c) {}
};
}  // namespace gdt

using namespace arx;

// the pieces of the reference's Context / Camera that full_render reads
struct Camera {
    glm::vec3 Position;
    float globalAngle;
};
struct DemoContext {
    AudioRenderer* renderer;
    OptixModel* model;
    Sphere* sphere;
    Camera* camera;
    std::vector<float>* audio;
    float* out_left;
    float* out_right;
};
static DemoContext Context;
static std::mutex audio_critical_section;

// main.cpp:40-67, unchanged but for the Context accessors
void full_render(bool isLive, std::mutex* output_buffer_mutex) {
    AudioRenderer* renderer = Context.renderer;
    OptixModel* scene = Context.model;
    Sphere sphere = *Context.sphere;
    Camera camera = *Context.camera;
    gdt::vec3f camera_central_point = gdt::vec3f(camera.Position.x, camera.Position.y, camera.Position.z);

    if (!isLive) {
        size_t len_of_audio = Context.audio->size();
        size_t size_of_audio = sizeof(float) * len_of_audio;
        float* outputBuffer_left = Context.out_left;
        float* outputBuffer_right = Context.out_right;
        audio_critical_section.lock();
        renderer->full_render_cycle(output_buffer_mutex, sphere, scene, camera_central_point, camera.globalAngle,
                                    Context.audio->data(), size_of_audio, outputBuffer_left, outputBuffer_right);
        audio_critical_section.unlock();
    } else {
        audio_critical_section.lock();
        placeReceiver(sphere, scene, camera_central_point, camera.globalAngle);
        renderer->setSphereCenterInOptix(glm::vec3(camera_central_point.x, camera_central_point.y, camera_central_point.z));
        renderer->render();
        audio_critical_section.unlock();
    }
}

static void write_raw(const std::string& path, const void* data, size_t bytes) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(data, 1, bytes, f) != bytes) {
        std::fprintf(stderr, "cannot write %s\n", path.c_str());
        std::exit(2);
    }
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr,
                     "usage: main_style_demo config.json leftHalf.obj rightHalf.obj out_dir angle_deg [frames_in_flight]\n");
        return 2;
    }
    const std::string out = argv[4];
    try {
        const arx_app_config cfg = loadConfig(argv[1]);
        OptixModel model{loadOBJ(cfg.scene_file_path)};
        HalfSphere left = loadHalfSphere(argv[2], true), right = loadHalfSphere(argv[3], false);
        Sphere sphere(&left, &right);
        Wav wav = loadWav(cfg.audio_file_path);
        // Context.cpp:228-231: new AudioRenderer(model, ir_length_in_seconds, sample_rate, materials, rays)
        AudioRenderer* renderer = new AudioRenderer(&model, cfg.ir_length_in_seconds, wav.sample_rate,
                                                    configMaterials(cfg),
                                                    gdt::vec3f(cfg.rays[0], cfg.rays[1], cfg.rays[2]));
        if (argc > 6) renderer->setFramesInFlight(std::atoi(argv[6]));  // not in main.cpp: the renderer mode
        renderer->setMonoOutput(cfg.mono != 0);
        renderer->setBasePower(cfg.base_power);
        renderer->setThresholds(cfg.ray_energy_threshold, cfg.ray_max_bounces);
        renderer->set_hrtf_absorption_rate(cfg.hrtf_absorption_rate);
        renderer->setEmitterPosInOptix(
            glm::vec3(cfg.initial_emitter_pos[0], cfg.initial_emitter_pos[1], cfg.initial_emitter_pos[2]));
        Camera camera{glm::vec3(cfg.initial_receiver_pos[0], cfg.initial_receiver_pos[1], cfg.initial_receiver_pos[2]),
                      (float)std::atof(argv[5])};
        std::vector<float> outL(wav.samples[0].size()), outR(wav.samples[0].size());
        Context = DemoContext{renderer, &model, &sphere, &camera, &wav.samples[0], outL.data(), outR.data()};
        std::mutex output_buffer_mutex;
        std::vector<float> irl(renderer->irLength()), irr(renderer->irLength());

        full_render(false, &output_buffer_mutex);  // file mode
        renderer->getIR(irl.data(), irr.data());
        write_raw(out + "/ir_file_left.f32", irl.data(), irl.size() * 4);
        write_raw(out + "/ir_file_right.f32", irr.data(), irr.size() * 4);
        write_raw(out + "/conv_left.f32", outL.data(), outL.size() * 4);
        write_raw(out + "/conv_right.f32", outR.data(), outR.size() * 4);

        camera.Position = glm::vec3(camera.Position.x + 0.5f, camera.Position.y, camera.Position.z - 0.25f);
        camera.globalAngle += 30.0f;
        full_render(true, &output_buffer_mutex);  // live mode, the camera moved and turned
        renderer->getIR(irl.data(), irr.data());
        write_raw(out + "/ir_live_left.f32", irl.data(), irl.size() * 4);
        write_raw(out + "/ir_live_right.f32", irr.data(), irr.size() * 4);
        const arx_stats st = renderer->stats();
        std::printf("queries %llu receiver_hits %llu\n", (unsigned long long)st.queries,
                    (unsigned long long)st.receiver_hits);
        delete renderer;
    } catch (const Error& e) {
        std::fprintf(stderr, "arx error: %s\n", e.what());
        return 1;
    }
    return 0;
}
