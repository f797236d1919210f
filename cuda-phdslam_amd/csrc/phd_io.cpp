/*
 * phd_io.cpp — SURVEY.md §8(f) rank 3: the reference's data loaders and its
 * per-step log writer, host-only (no GPU, no Boost).
 *
 * Loaders (src/main.cpp:147-245):
 *   loadTimestamps    :147-167  one value per line
 *   loadControls      :169-190  header line, then "v_encoder alpha" per line
 *   loadMeasurements  :221-245  header line, then one time step per line of
 *                               "range bearing label" triples (parseMeasurements
 *                               :192-208)
 * The reference's loops push one element past the data (the failed extraction
 * of the read at EOF, and of a trailing separator inside a measurement line:
 * "TODO: sloppily remove the last invalid measurement", :206-207) with
 * uninitialised fields; these loaders stop at the last complete record
 * instead.  The files the reference ships (python/controls_synth.txt,
 * python/measurements_synth.txt) have no header line and separate with ", " /
 * pairs without labels, which the reference's loaders mis-parse (SURVEY.md
 * §8(f)); PHD_IO_* flags select the format explicitly.
 *
 * Writer (writeLog, src/main.cpp:848-954; declared but never called by the
 * reference): state_estimateNNNNN.log, appended, seven lines — expected pose
 * (6 fields), static map (weight mean[2] cov[4] per component), dynamic map
 * (empty: the static feature model), particle log-weights (repeated
 * n_predict_particles times at t = 0), particle poses (likewise), resample
 * indices, cardinality distribution (maxCardinality + 1 values, "0" when the
 * filter is not CPHD).  Numbers go through std::ostream with its default
 * formatting, exactly as the reference's fstream << float does, so the bytes
 * match for the same values.
 */
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <string>
#include <vector>

#include "phd_capi.h"
#include "phd_io.h"

namespace {

/* numbers of one line: separators are whitespace, plus ',' when `commas` */
std::vector<double> numbers(std::string line, bool commas, bool* complete) {
    if (commas)
        for (char& ch : line)
            if (ch == ',') ch = ' ';
    std::vector<double> v;
    const char* p = line.c_str();
    bool ok = true;
    while (*p) {
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') p++;
        if (!*p) break;
        char* end = nullptr;
        errno = 0;
        const double x = strtod(p, &end);
        if (end == p) {  // not a number: the reference's extraction stops here
            ok = false;
            break;
        }
        v.push_back(x);
        p = end;
    }
    if (complete) *complete = ok;
    return v;
}

bool read_lines(const char* path, int flags, std::vector<std::string>& lines) {
    std::ifstream f(path);
    if (!f.is_open()) return false;
    std::string line;
    bool first = true;
    while (std::getline(f, line)) {
        if (first && (flags & PHD_IO_HEADER)) {  // "skip header line" (main.cpp:176-177, :229-230)
            first = false;
            continue;
        }
        first = false;
        if (flags & PHD_IO_COMMENTS) {
            const size_t b = line.find_first_not_of(" \t");
            if (b != std::string::npos && (line[b] == '%' || line[b] == '#')) continue;
        }
        lines.push_back(line);
    }
    // the read at EOF (an empty last line) is not a record
    while (!lines.empty() && lines.back().find_first_not_of(" \t\r") == std::string::npos) lines.pop_back();
    return true;
}

}  // namespace

extern "C" {

int phd_load_timestamps(const char* path, double* out, int cap, int* n) {
    if (!path || !n || cap < 0 || (cap > 0 && !out)) return PHD_E_ARG;
    std::vector<std::string> lines;
    if (!read_lines(path, 0, lines)) return PHD_E_ARG;
    int k = 0;
    for (const auto& l : lines) {
        const auto v = numbers(l, false, nullptr);
        if (v.empty()) continue;
        if (k < cap) out[k] = v[0];
        k++;
    }
    *n = k;
    return k > cap ? PHD_E_CAPACITY : PHD_OK;
}

int phd_load_controls(const char* path, int flags, phd_ackerman_control* out, int cap, int* n) {
    if (!path || !n || cap < 0 || (cap > 0 && !out)) return PHD_E_ARG;
    std::vector<std::string> lines;
    if (!read_lines(path, flags, lines)) return PHD_E_ARG;
    int k = 0;
    for (const auto& l : lines) {
        const auto v = numbers(l, (flags & PHD_IO_COMMAS) != 0, nullptr);
        if (v.size() < 2) continue;  // `ss >> u.v_encoder >> u.alpha` (main.cpp:183)
        if (k < cap) {
            out[k].v_encoder = (float)v[0];
            out[k].alpha = (float)v[1];
        }
        k++;
    }
    *n = k;
    return k > cap ? PHD_E_CAPACITY : PHD_OK;
}

int phd_load_measurements(const char* path, int flags, phd_measurement* out, long cap, int* offsets, int max_steps,
                          int* n_steps) {
    if (!path || !n_steps || cap < 0 || max_steps < 0 || (cap > 0 && !out) || !offsets)
        return PHD_E_ARG;
    std::vector<std::string> lines;
    if (!read_lines(path, flags, lines)) return PHD_E_ARG;
    const size_t w = (flags & PHD_IO_PAIRS) ? 2 : 3;
    long k = 0;
    int s = 0;
    bool over = false;
    for (const auto& l : lines) {
        if (s <= max_steps) offsets[s] = (int)k;
        const auto v = numbers(l, (flags & PHD_IO_COMMAS) != 0, nullptr);
        // parseMeasurements (main.cpp:192-208): range bearing label per measurement
        for (size_t i = 0; i + w <= v.size(); i += w) {
            if (k < cap) {
                out[k].range = (float)v[i];
                out[k].bearing = (float)v[i + 1];
                out[k].label = w == 3 ? (int)v[i + 2] : 0;
            } else {
                over = true;
            }
            k++;
        }
        s++;
    }
    if (s <= max_steps) offsets[s] = (int)k;
    *n_steps = s;
    if (s > max_steps) return PHD_E_CAPACITY;
    return over ? PHD_E_CAPACITY : PHD_OK;
}

int phd_write_state_log(const char* dir, int t, const phd_pose* expected_pose, const phd_gaussian2d* map,
                        long n_map, const float* log_weights, const phd_pose* poses, int n, const int* resample_idx,
                        const float* cn, int max_cardinality, int filter_type, int n_predict_particles) {
    if (t < 0 || !expected_pose || n < 0 || n_map < 0 || (n_map > 0 && !map) || (n > 0 && (!log_weights || !poses)) ||
        max_cardinality < 0 || (filter_type == 1 && !cn))
        return PHD_E_ARG;
    std::ostringstream name;
    if (dir && *dir) {
        name << dir;
        if (name.str().back() != '/') name << '/';
    }
    name << "state_estimate" << std::setfill('0') << std::setw(5) << t << ".log";
    std::fstream f(name.str().c_str(), std::fstream::out | std::fstream::app);
    if (!f.is_open()) return PHD_E_ARG;
    const phd_pose& e = *expected_pose;
    f << e.px << " " << e.py << " " << e.ptheta << " " << e.vx << " " << e.vy << " " << e.vtheta << " " << std::endl;
    for (long k = 0; k < n_map; k++) {
        f << map[k].weight << " ";
        for (int i = 0; i < 2; i++) f << map[k].mean[i] << " ";
        for (int i = 0; i < 4; i++) f << map[k].cov[i] << " ";
    }
    f << std::endl;
    f << std::endl;  // dynamic map: none (static feature model)
    const int times = (t == 0 && n_predict_particles > 1) ? n_predict_particles : 1;  // main.cpp:906-910
    for (int r = 0; r < times; r++)
        for (int k = 0; k < n; k++) f << log_weights[k] << " ";
    f << std::endl;
    for (int r = 0; r < times; r++)
        for (int k = 0; k < n; k++) {
            const phd_pose& s = poses[k];
            f << s.px << " " << s.py << " " << s.ptheta << " " << s.vx << " " << s.vy << " " << s.vtheta << " ";
        }
    f << std::endl;
    for (int k = 0; k < n; k++) f << (resample_idx ? resample_idx[k] : k) << " ";
    f << std::endl;
    for (int k = 0; k <= max_cardinality; k++) {
        if (filter_type == 1)
            f << cn[k] << " ";
        else
            f << "0 ";
    }
    f << std::endl;
    f.close();
    return f.fail() ? PHD_E_ARG : PHD_OK;
}

}  // extern "C"
