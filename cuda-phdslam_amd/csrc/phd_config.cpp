/*
 * phd_config.cpp — the reference's cfg/config.cfg surface without Boost.
 *
 * Restates loadConfig (main.cpp:956-1073): boost::program_options config-file
 * syntax ("key = value", '#' starts a comment anywhere on a line, section
 * headers ignored), the same key names and defaults, then
 * clutterDensity = clutterRate / (2 * maxBearing * maxRange) (main.cpp:1065).
 *
 * Deviation: initial_vz / initial_vroll /
 * initial_vpitch bind vz0 / vroll0 / vpitch0 here; the reference binds them to
 * vy0 / vyaw0 / vyaw0 (main.cpp:970-972).
 */
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>

#include "phd_capi.h"

namespace {

enum Kind { KF, KI, KB, KS, KIGNORE };

struct Key {
    Kind kind;
    size_t off;
};

#define F(name, field) {name, {KF, offsetof(phd_slam_config, field)}}
#define I(name, field) {name, {KI, offsetof(phd_slam_config, field)}}
#define B(name, field) {name, {KB, offsetof(phd_slam_config, field)}}

const std::map<std::string, Key>& keys() {
    static const std::map<std::string, Key> k = {
        B("debug", debug),
        F("initial_x", x0), F("initial_y", y0), F("initial_z", z0),
        F("initial_roll", roll0), F("initial_pitch", pitch0), F("initial_yaw", yaw0),
        F("initial_vx", vx0), F("initial_vy", vy0), F("initial_vz", vz0),
        F("initial_vroll", vroll0), F("initial_vpitch", vpitch0), F("initial_vyaw", vyaw0),
        B("follow_trajectory", followTrajectory),
        I("motion_type", motionType),
        F("acc_x", ax), F("acc_y", ay), F("acc_z", az),
        F("acc_roll", aroll), F("acc_pitch", apitch), F("acc_yaw", ayaw),
        F("dt", dt),
        F("max_bearing", maxBearing), F("min_range", minRange), F("max_range", maxRange),
        F("std_bearing", stdBearing), F("std_range", stdRange),
        F("clutter_rate", clutterRate), F("pd", pd), F("ps", ps),
        I("n_particles", n_particles), I("n_predict_particles", nPredictParticles),
        F("resample_threshold", resampleThresh), I("subdivide_predict", subdividePredict),
        F("birth_weight", birthWeight), F("birth_noise_factor", birthNoiseFactor),
        B("gate_births", gateBirths), B("gate_measurements", gateMeasurements),
        F("gate_threshold", gateThreshold),
        I("feature_model", featureModel),
        F("min_expected_feature_weight", minExpectedFeatureWeight),
        F("min_separation", minSeparation), I("max_features", maxFeatures),
        F("min_feature_weight", minFeatureWeight), I("particle_weighting", particleWeighting),
        I("daughter_mixture_type", daughterMixtureType), I("n_samples", nSamples),
        I("max_cardinality", maxCardinality), I("filter_type", filterType),
        I("map_estimate", mapEstimate), I("cphd_disttype", cphdDistType), F("nu", nu),
        I("distance_metric", distanceMetric),
        F("h", h), F("l", l), F("a", a), F("b", b),
        F("std_encoder", stdEncoder), F("std_alpha", stdAlpha),
        F("std_vx_features", stdVxMap), F("std_vy_features", stdVyMap),
        F("std_ax_features", stdAxMap), F("std_ay_features", stdAyMap),
        F("cov_vx_birth", covVxBirth), F("cov_vy_birth", covVyBirth),
        F("std_u", stdU), F("std_v", stdV), F("disparity_birth", disparityBirth),
        I("image_width", imageWidth), I("image_height", imageHeight),
        F("std_d_birth", stdDBirth), F("fx", fx), F("fy", fy), F("u0", u0), F("v0", v0),
        I("particles_per_feature", particlesPerFeature),
        F("tau", tau), F("beta", beta),
        B("labeled_measurements", labeledMeasurements),
        I("max_time_steps", maxSteps),
        B("save_all_maps", saveAllMaps), B("save_prediction", savePrediction),
        {"data_directory", {KS, 0}},
        {"n_steps", {KIGNORE, 0}},
    };
    return k;
}
#undef F
#undef I
#undef B

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

bool parse_bool(const std::string& v, bool* out) {
    std::string t;
    for (char ch : v) t += (char)std::tolower((unsigned char)ch);
    if (t == "1" || t == "true" || t == "yes" || t == "on") {
        *out = true;
        return true;
    }
    if (t == "0" || t == "false" || t == "no" || t == "off") {
        *out = false;
        return true;
    }
    return false;
}

}  // namespace

extern "C" {

int phd_config_defaults(phd_slam_config* c) {
    if (!c) return PHD_E_ARG;
    std::memset(c, 0, sizeof(*c));
    // defaults of loadConfig (main.cpp:961-1048)
    c->debug = false;
    c->motionType = 1;
    c->ax = 0.5f;
    c->ay = 0.f;
    c->az = 0.f;
    c->aroll = 0.0087f;
    c->apitch = 0.0087f;
    c->ayaw = 0.0087f;
    c->dt = 0.1f;
    c->maxBearing = (float)M_PI;
    c->minRange = 0.f;
    c->maxRange = 20.f;
    c->stdBearing = 0.0524f;
    c->stdRange = 1.0f;
    c->clutterRate = 15.f;
    c->pd = 0.98f;
    c->ps = 0.98f;
    c->n_particles = 512;
    c->nPredictParticles = 1;
    c->resampleThresh = 0.15f;
    c->subdividePredict = 1;
    c->birthWeight = 0.05f;
    c->birthNoiseFactor = 1.5f;
    c->gateBirths = true;
    c->gateMeasurements = true;
    c->gateThreshold = 10.f;
    c->featureModel = 0;
    c->minExpectedFeatureWeight = 0.33f;
    c->minSeparation = 5.f;
    c->maxFeatures = 100;
    c->minFeatureWeight = 0.00001f;
    c->particleWeighting = 1;
    c->daughterMixtureType = 0;
    c->nSamples = 50;
    c->maxCardinality = 256;
    c->filterType = 1;
    c->mapEstimate = 1;
    c->cphdDistType = 0;
    c->nu = 1.f;
    c->distanceMetric = 0;
    c->stdU = 1.f;
    c->stdV = 1.f;
    c->disparityBirth = 1000.f;
    c->imageWidth = 600;
    c->imageHeight = 480;
    c->stdDBirth = 300.f;
    c->fx = 1000.f;
    c->fy = 1000.f;
    c->u0 = 512.f;
    c->v0 = 384.f;
    c->particlesPerFeature = 100;
    c->tau = 0.f;
    c->beta = 1.f;
    c->labeledMeasurements = false;
    c->maxSteps = 10000;
    c->saveAllMaps = false;
    c->savePrediction = false;
    c->clutterDensity = c->clutterRate / (2 * c->maxBearing * c->maxRange);
    return PHD_OK;
}

int phd_config_load(const char* path, phd_slam_config* c, char* data_dir, int data_dir_cap) {
    if (!path || !c) return PHD_E_ARG;
    std::ifstream f(path);
    if (!f) return PHD_E_ARG;
    phd_config_defaults(c);
    std::string line;
    unsigned char* base = reinterpret_cast<unsigned char*>(c);
    while (std::getline(f, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty() || line[0] == '[') continue;
        const size_t eq = line.find('=');
        if (eq == std::string::npos) return PHD_E_ARG;
        const std::string k = trim(line.substr(0, eq));
        const std::string v = trim(line.substr(eq + 1));
        auto it = keys().find(k);
        if (it == keys().end()) return PHD_E_ARG;  // boost rejects unregistered options
        const Key& key = it->second;
        char* end = nullptr;
        switch (key.kind) {
            case KF: {
                float x = std::strtof(v.c_str(), &end);
                if (end == v.c_str()) return PHD_E_ARG;
                std::memcpy(base + key.off, &x, sizeof(float));
                break;
            }
            case KI: {
                long x = std::strtol(v.c_str(), &end, 10);
                if (end == v.c_str()) return PHD_E_ARG;
                int xi = (int)x;
                std::memcpy(base + key.off, &xi, sizeof(int));
                break;
            }
            case KB: {
                bool x;
                if (!parse_bool(v, &x)) return PHD_E_ARG;
                std::memcpy(base + key.off, &x, sizeof(bool));
                break;
            }
            case KS:
                if (data_dir && data_dir_cap > 0) {
                    std::strncpy(data_dir, v.c_str(), (size_t)data_dir_cap - 1);
                    data_dir[data_dir_cap - 1] = 0;
                }
                break;
            case KIGNORE:
                break;
        }
    }
    c->clutterDensity = c->clutterRate / (2 * c->maxBearing * c->maxRange);  // main.cpp:1065-1066
    return PHD_OK;
}

}  // extern "C"
