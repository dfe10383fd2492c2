// export_demo -- a main.cpp-style caller of the C++ AudioRenderer shim (include/arx_audio_renderer.hpp)
// on the GPU: the reference's export_audio flow (R/prebuild/obj_raytracer/main.cpp:653-718) plus one
// mic callback (audioHandlerWithMic, main.cpp:99-135), through libarx.so's group API.
//
//   export_demo config.json leftHalf.obj rightHalf.obj out_dir devices(e.g. "0" or "0,0,0,0") [dumps]
//
// Loads config.json (Context::loadContext), the OBJ scene and the receiver halves (loadOBJ,
// HalfSphere), the WAV (AudioFile), renders, convolves the file (convoluteAudioFile), runs one
// 4096-frame live block into a CircularBuffer (convoluteLiveInput), and writes raw results to
// out_dir for tests/test_gpu_shim.py to compare with the CPU oracle:
//   ir_left.f32 ir_right.f32 conv_left.f32 conv_right.f32 live.f64, and a stats line on stdout.
// With "dumps", it then replays key P of main.cpp:317-322 inside out_dir: render, set both write
// flags, render again (writes output_ir_{left,right}.txt, AudioRenderer.cpp:525-567), convolve
// (writes output_convolute_{left,right}.txt, :720-744); a further render + convolve must write
// nothing (the flags reset after one write).
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <sstream>
#include <string>
#include <vector>

#include "arx_audio_renderer.hpp"
#include "arx_circular_buffer.hpp"

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
        std::fprintf(stderr, "usage: export_demo config.json leftHalf.obj rightHalf.obj out_dir devices\n");
        return 2;
    }
    const std::string out = argv[4];
    std::vector<int32_t> devices;
    {
        std::stringstream ss(argv[5]);
        std::string tok;
        while (std::getline(ss, tok, ',')) devices.push_back(std::atoi(tok.c_str()));
    }
    try {
        // Context::loadContext (Context.cpp:15-236)
        const arx_app_config cfg = arx::loadConfig(argv[1]);
        const std::vector<arx::Mesh> model = arx::loadOBJ(cfg.scene_file_path);
        const arx::Mesh left = arx::loadHalfSphere(argv[2], true);
        const arx::Mesh right = arx::loadHalfSphere(argv[3], false);
        arx::Wav wav = arx::loadWav(cfg.audio_file_path);
        const arx::Vec3 rays = {cfg.rays[0], cfg.rays[1], cfg.rays[2]};
        arx::AudioRenderer r(model, cfg.ir_length_in_seconds, wav.sample_rate, arx::configMaterials(cfg), rays, devices);
        r.setReceiverModel(left, right);
        // the setters main.cpp calls before rendering (main.cpp:411-418, 548-553)
        r.setMonoOutput(cfg.mono != 0);
        r.setBasePower(cfg.base_power);
        r.setThresholds(cfg.ray_energy_threshold, cfg.ray_max_bounces);
        r.set_hrtf_absorption_rate(cfg.hrtf_absorption_rate);
        r.setEmitterPosInOptix({cfg.initial_emitter_pos[0], cfg.initial_emitter_pos[1], cfg.initial_emitter_pos[2]});
        r.setSphereCenterInOptix({cfg.initial_receiver_pos[0], cfg.initial_receiver_pos[1], cfg.initial_receiver_pos[2]});
        double render_ms = 0.0;
        r.render(&render_ms);
        std::vector<float> irl(r.irLength()), irr(r.irLength());
        r.getIR(irl.data(), irr.data());
        write_raw(out + "/ir_left.f32", irl.data(), irl.size() * 4);
        write_raw(out + "/ir_right.f32", irr.data(), irr.size() * 4);
        // export_audio: convolve channel 0 of the file (main.cpp:682-684)
        std::vector<float>& x = wav.samples[0];
        std::vector<float> cl(x.size()), cr(x.size());
        double conv_ms = 0.0, proc_ms = 0.0;
        r.convoluteAudioFile(x.data(), x.size() * sizeof(float), cl.data(), cr.data(), &conv_ms, &proc_ms);
        write_raw(out + "/conv_left.f32", cl.data(), cl.size() * 4);
        write_raw(out + "/conv_right.f32", cr.data(), cr.size() * 4);
        // one mic callback: 4096 f64 frames -> CircularBuffer(44100 * ir_sec) -> get_and_reset(2 * 4096)
        std::vector<double> mic(4096);
        for (size_t i = 0; i < mic.size(); ++i) mic[i] = (double)x[i % x.size()];
        arx::CircularBuffer<double> cb((size_t)44100 * cfg.ir_length_in_seconds);
        r.convoluteLiveInput(mic.data(), mic.size() * sizeof(double), &cb);
        const std::vector<double> live = cb.get_and_reset(2 * mic.size());
        write_raw(out + "/live.f64", live.data(), live.size() * 8);
        if (argc > 6 && std::string(argv[6]) == "dumps") {
            if (chdir(out.c_str()) != 0) return 2;
            r.render();
            r.set_write_ir_to_file_flag(true);
            r.set_write_output_to_file_flag(true);
            r.render();
            r.convoluteAudioFile(x.data(), x.size() * sizeof(float), cl.data(), cr.data());
            const char* dumps[4] = {"output_ir_left.txt", "output_ir_right.txt", "output_convolute_left.txt",
                                    "output_convolute_right.txt"};
            for (const char* f : dumps)
                if (std::rename(f, (std::string(f) + ".first").c_str()) != 0) {
                    std::fprintf(stderr, "%s was not written\n", f);
                    return 3;
                }
            r.render();
            r.convoluteAudioFile(x.data(), x.size() * sizeof(float), cl.data(), cr.data());
            for (const char* f : dumps)
                if (access(f, F_OK) == 0) {
                    std::fprintf(stderr, "%s written twice (the flag did not reset)\n", f);
                    return 4;
                }
            std::printf("dumps ok\n");
        }
        const arx_stats st = r.stats();
        std::printf("queries %llu receiver_hits %llu misses %llu gpus %d render_ms %.3f conv_ms %.3f\n",
                    (unsigned long long)st.queries, (unsigned long long)st.receiver_hits, (unsigned long long)st.misses,
                    r.gpuCount(), render_ms, conv_ms);
    } catch (const arx::Error& e) {
        std::fprintf(stderr, "arx error: %s\n", e.what());
        return 1;
    }
    return 0;
}
