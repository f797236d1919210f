/*
 * phdslam_run.cpp — the run_synth driver (main.cpp:1075-1322) rebuilt on the
 * drop-in API (include/phdfilter.h) or, with --device-loop, on the
 * device-resident C-ABI loop (phd_step).
 *
 *   phdslam_run <config.cfg> [--data DIR] [--steps N] [--triples] [--device-loop]
 *
 * Inputs (DATA = data_directory of the cfg, or --data):
 *   DATA/measurements.txt  one time step per line, range/bearing pairs
 *                          (--triples: range bearing label, the format
 *                          parseMeasurements reads, main.cpp:190-205)
 *   DATA/controls.txt      one "v_encoder alpha" per line ('%' header lines and
 *                          ',' separators accepted)
 * Lines starting with '%' are headers.  Step n uses measurements[n] and, for
 * n > 0, controls[n-1] (main.cpp:1233-1234).
 */
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "phd_capi.h"
#include "phdfilter.h"

static std::vector<std::vector<double>> read_rows(const std::string& path) {
    std::vector<std::vector<double>> rows;
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        if (!line.empty() && line[0] == '%') continue;
        for (char& ch : line)
            if (ch == ',') ch = ' ';
        std::stringstream ss(line);
        std::vector<double> v;
        double x;
        while (ss >> x) v.push_back(x);
        rows.push_back(v);
    }
    while (!rows.empty() && rows.back().empty()) rows.pop_back();
    return rows;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <config.cfg> [--data DIR] [--steps N] [--triples] [--device-loop]\n", argv[0]);
        return 1;
    }
    SlamConfig config;
    char data_dir[4096] = "";
    if (phd_config_load(argv[1], &config, data_dir, sizeof(data_dir)) != PHD_OK) {
        fprintf(stderr, "Unable to load config file: %s\n", argv[1]);
        return 1;
    }
    std::string data = data_dir;
    int n_steps = -1;
    bool triples = false, device_loop = false;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--data") && i + 1 < argc) data = argv[++i];
        else if (!strcmp(argv[i], "--steps") && i + 1 < argc) n_steps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--triples")) triples = true;
        else if (!strcmp(argv[i], "--device-loop")) device_loop = true;
    }
    if (!data.empty() && data.back() != '/') data += '/';
    const auto zrows = read_rows(data + "measurements.txt");
    const auto urows = read_rows(data + "controls.txt");
    std::vector<measurementSet> allZ;
    for (const auto& r : zrows) {
        measurementSet Z;
        const size_t w = triples ? 3 : 2;
        for (size_t k = 0; k + w - 1 < r.size(); k += w) {
            RangeBearingMeasurement z;
            z.range = (float)r[k];
            z.bearing = (float)r[k + 1];
            z.label = triples ? (int)r[k + 2] : 0;
            Z.push_back(z);
        }
        allZ.push_back(Z);
    }
    int nSteps = (int)allZ.size();
    if (n_steps > 0 && n_steps < nSteps) nSteps = n_steps;
    printf("loaded %zu measurement steps, %zu controls; running %d steps with %d particles\n", allZ.size(),
           urows.size(), nSteps, config.n_particles);

    setDeviceConfig(config);
    initRandomNumberGenerators();
    const int N = config.n_particles;
    SynthSLAM particles(N);
    for (int n = 0; n < N; n++) {
        ConstantVelocityState& s = particles.states[n];
        s.px = config.x0;
        s.py = config.y0;
        s.ptheta = config.yaw0;
        s.vx = config.vx0;
        s.vy = config.vy0;
        s.vtheta = config.vyaw0;
    }
    particles.weights.assign(N, -log((float)N));

    auto t0 = std::chrono::steady_clock::now();
    if (!device_loop) {
        ConstantVelocityState expectedPose;
        vector<REAL> cn;
        for (int n = 0; n < nSteps; n++) {
            const measurementSet& ZZ = allZ[n];
            AckermanControl u{0.f, 0.f};
            if (n > 0 && n - 1 < (int)urows.size() && urows[n - 1].size() >= 2) {
                u.v_encoder = (float)urows[n - 1][0];
                u.alpha = (float)urows[n - 1][1];
            }
            if (n > 0)
                for (int i = 0; i < config.subdividePredict; i++) {
                    if (config.motionType == CV_MOTION)
                        phdPredict(particles);
                    else
                        phdPredict(particles, u);
                }
            if (!ZZ.empty()) phdUpdateSynth(particles, ZZ);
            recoverSlamState(particles, expectedPose, cn);
            float nEff = 0;
            for (int i = 0; i < particles.n_particles; i++) nEff += exp(2 * particles.weights[i]);
            nEff = 1.0 / nEff / particles.n_particles;
            size_t ncomp = 0;
            for (const auto& m : particles.maps_static) ncomp += m.size();
            printf("step %5d |Z|=%3zu nEff=%.4f pose=(%.3f, %.3f, %.4f) mean map size %.1f\n", n, ZZ.size(), nEff,
                   expectedPose.px, expectedPose.py, expectedPose.ptheta, (double)ncomp / particles.n_particles);
            if (nEff <= config.resampleThresh && !ZZ.empty()) particles = resampleParticles(particles, N, (uint64_t)n);
            if (std::isnan(nEff)) {
                printf("nan weights detected! exiting...\n");
                break;
            }
        }
    } else {
        phd_ctx* ctx = nullptr;
        phd_capacity cap{};
        cap.map_capacity = 2048;
        cap.candidate_capacity = 3072;
        if (phd_ctx_create(&ctx, 0, N, &cap) != PHD_OK || phd_set_config(ctx, &config) != PHD_OK) {
            fprintf(stderr, "phd_ctx_create: %s\n", phd_last_error());
            return 1;
        }
        std::vector<int> offs(N + 1, 0);
        if (phd_load_particles(ctx, N, particles.states.data(), particles.weights.data(), nullptr, offs.data()) !=
            PHD_OK) {
            fprintf(stderr, "phd_load_particles: %s\n", phd_last_error());
            return 1;
        }
        for (int n = 0; n < nSteps; n++) {
            AckermanControl u{0.f, 0.f};
            if (n > 0 && n - 1 < (int)urows.size() && urows[n - 1].size() >= 2) {
                u.v_encoder = (float)urows[n - 1][0];
                u.alpha = (float)urows[n - 1][1];
            }
            if (phd_set_measurements(ctx, allZ[n].data(), (int)allZ[n].size()) != PHD_OK ||
                phd_step(ctx, &u, n > 0, (uint64_t)n, nullptr, nullptr) != PHD_OK) {
                fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                return 1;
            }
        }
        ConstantVelocityState ep;
        int mi;
        phd_expected_pose(ctx, &ep, &mi);
        printf("final expected pose (%.3f, %.3f, %.4f), MAP particle %d\n", ep.px, ep.py, ep.ptheta, mi);
        phd_ctx_destroy(ctx);
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%d steps in %.3f s (%.1f steps/s)\n", nSteps, secs, nSteps / secs);
    return 0;
}
