// config.cc — INI loading and validation (see config.h).
#include "config.h"

#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <climits>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "common.h"

namespace switchml {

namespace {

std::string trim(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && std::isspace((unsigned char)s[b])) b++;
    while (e > b && std::isspace((unsigned char)s[e - 1])) e--;
    return s.substr(b, e - b);
}

bool parse_bool(const std::string& v) {
    std::string l = v;
    std::transform(l.begin(), l.end(), l.begin(), ::tolower);
    if (l == "true" || l == "1" || l == "yes" || l == "on") return true;
    if (l == "false" || l == "0" || l == "no" || l == "off") return false;
    throw SwitchMLFatal("invalid boolean '" + v + "'");
}

template <typename T>
T parse_uint(const std::string& key, const std::string& v, unsigned long long max) {
    size_t pos = 0;
    unsigned long long x = std::stoull(v, &pos, 0);
    if (pos != v.size() || x > max) throw SwitchMLFatal("invalid value '" + v + "' for " + key);
    return (T)x;
}

}  // namespace

bool Config::LoadFromString(const std::string& ini) {
    std::istringstream in(ini);
    std::string line, section;
    while (std::getline(in, line)) {
        auto hash = line.find_first_of("#;");
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty()) continue;
        if (line.front() == '[' && line.back() == ']') {
            section = trim(line.substr(1, line.size() - 2));
            continue;
        }
        auto eq = line.find('=');
        if (eq == std::string::npos) throw SwitchMLFatal("malformed config line '" + line + "'");
        std::string key = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
        std::string full = section.empty() ? key : section + "." + key;
        GeneralConfig& g = general_;
        if (full == "general.rank") g.rank = parse_uint<uint16_t>(full, val, 0xffff);
        else if (full == "general.num_workers") g.num_workers = parse_uint<uint16_t>(full, val, 0xffff);
        else if (full == "general.num_worker_threads") g.num_worker_threads = parse_uint<uint16_t>(full, val, 0xffff);
        else if (full == "general.max_outstanding_packets") g.max_outstanding_packets = parse_uint<uint32_t>(full, val, 0xffffffffull);
        else if (full == "general.packet_numel") g.packet_numel = parse_uint<uint64_t>(full, val, ~0ull);
        else if (full == "general.backend") g.backend = val;
        else if (full == "general.scheduler") g.scheduler = val;
        else if (full == "general.prepostprocessor") g.prepostprocessor = val;
        else if (full == "general.instant_job_completion") g.instant_job_completion = parse_bool(val);
        else if (full == "general.controller_ip") g.controller_ip_str = val;
        else if (full == "general.controller_port") g.controller_port = parse_uint<uint16_t>(full, val, 0xffff);
        else if (full == "backend.dummy.bandwidth") backend_.dummy.bandwidth = std::stof(val);
        else if (full == "backend.dummy.process_packets") backend_.dummy.process_packets = parse_bool(val);
        else if (full == "backend.dummy.fail_worker_thread") backend_.dummy.fail_worker_thread = std::stoi(val);
        else if (full == "backend.dummy.stall_worker_thread") backend_.dummy.stall_worker_thread = std::stoi(val);
        else if (full == "backend.dummy.stall_ms") backend_.dummy.stall_ms = parse_uint<uint32_t>(full, val, 60000ull);
        else if (full == "backend.hip.device") backend_.hip.device = std::stoi(val);
        else if (full == "backend.xgmi.session") backend_.xgmi.session = val;
        else if (full == "backend.xgmi.max_slice_numel") backend_.xgmi.max_slice_numel = parse_uint<uint64_t>(full, val, ~0ull);
        else if (full == "backend.xgmi.timeout_ms") backend_.xgmi.timeout_ms = parse_uint<uint64_t>(full, val, ~0ull);
        else if (full == "backend.xgmi.push") backend_.xgmi.push = parse_bool(val);
        else if (full == "backend.xgmi.fail_setup") backend_.xgmi.fail_setup = parse_bool(val);
        else if (full == "backend.hip.mode") backend_.hip.mode = val;
        else if (full == "backend.hip.packet_ring") backend_.hip.packet_ring = val;
        else if (full == "backend.hip.burst_server") backend_.hip.burst_server = parse_bool(val);
        else if (full == "backend.hip.batch_jobs") backend_.hip.batch_jobs = parse_uint<uint32_t>(full, val, 0xffffffffull);
        else if (full == "backend.hip.coalesce_us") backend_.hip.coalesce_us = parse_uint<uint32_t>(full, val, 1000000ull);
        else if (full == "backend.hip.vcl") backend_.hip.vcl = parse_bool(val);
        else fprintf(stderr, "[switchml] ignoring config key '%s' (not used by this build)\n", full.c_str());
    }
    return true;
}

bool Config::LoadFromFile(std::string path) {
    std::vector<std::string> candidates;
    if (!path.empty()) {
        candidates.push_back(path);
    } else {
        char host[HOST_NAME_MAX + 1] = {0};
        if (gethostname(host, sizeof(host)) != 0) throw SwitchMLFatal("gethostname failed");
        candidates = {"/etc/switchml.cfg", "switchml.cfg", std::string("switchml-") + host + ".cfg"};
    }
    for (const auto& c : candidates) {
        std::ifstream f(c);
        if (!f.good()) continue;
        std::stringstream ss;
        ss << f.rdbuf();
        return LoadFromString(ss.str());
    }
    return false;
}

void Config::Validate() {
    GeneralConfig& g = general_;
    if (g.num_worker_threads == 0) throw SwitchMLFatal("general.num_worker_threads must be >= 1");
    if (g.num_workers == 0) throw SwitchMLFatal("general.num_workers must be >= 1");
    if (g.packet_numel == 0) throw SwitchMLFatal("general.packet_numel must be >= 1");
    const uint64_t T = g.num_worker_threads;
    if (g.max_outstanding_packets / T == 0)
        throw SwitchMLFatal("max_outstanding_packets must be at least num_worker_threads");
    if (g.max_outstanding_packets % T != 0) {
        // Round to the nearest multiple of T (ties and below-equal go down), as config.cc:160-170.
        uint64_t lo = (g.max_outstanding_packets / T) * T, hi = lo + T;
        uint64_t pick = (g.max_outstanding_packets - lo > hi - g.max_outstanding_packets) ? hi : lo;
        fprintf(stderr, "[switchml] general.max_outstanding_packets %u is not divisible by %u; using %llu\n",
                g.max_outstanding_packets, (unsigned)T, (unsigned long long)pick);
        g.max_outstanding_packets = (uint32_t)pick;
    }
    if (g.scheduler != "fifo") throw SwitchMLFatal("'" + g.scheduler + "' is not a valid scheduler");
    if (g.backend != "dummy" && g.backend != "xgmi")
        throw SwitchMLFatal("'" + g.backend + "' is not a backend of this build (dummy | xgmi)");
    if (g.backend == "xgmi") {
        const std::string& s = backend_.xgmi.session;
        if (s.empty() || s.size() > 200 ||
            s.find_first_not_of("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_.") != std::string::npos)
            throw SwitchMLFatal("backend.xgmi.session must be a non-empty name of [A-Za-z0-9-_.]");
        if (g.rank >= g.num_workers) throw SwitchMLFatal("general.rank must be < general.num_workers");
        if (g.num_workers > 16 || g.num_worker_threads > 16)
            throw SwitchMLFatal("the xgmi backend supports up to 16 workers and 16 worker threads");
        if (g.prepostprocessor == "bypass") throw SwitchMLFatal("the xgmi backend needs the HIP pre/post-processor");
        if (backend_.xgmi.max_slice_numel == 0) throw SwitchMLFatal("backend.xgmi.max_slice_numel must be >= 1");
    }
    const std::string& m = backend_.hip.mode;
    if (m != "bulk" && m != "fused" && m != "packet") throw SwitchMLFatal("backend.hip.mode must be bulk|fused|packet");
    const std::string& r = backend_.hip.packet_ring;
    if (r != "device" && r != "pinned" && r != "pageable")
        throw SwitchMLFatal("backend.hip.packet_ring must be device|pinned|pageable");
}

std::string Config::ToString() const {
    std::ostringstream o;
    const GeneralConfig& g = general_;
    o << "[general]\nrank = " << g.rank << "\nnum_workers = " << g.num_workers
      << "\nnum_worker_threads = " << g.num_worker_threads
      << "\nmax_outstanding_packets = " << g.max_outstanding_packets << "\npacket_numel = " << g.packet_numel
      << "\nbackend = " << g.backend << "\nscheduler = " << g.scheduler
      << "\nprepostprocessor = " << g.prepostprocessor
      << "\ninstant_job_completion = " << (g.instant_job_completion ? "true" : "false")
      << "\ncontroller_ip = " << g.controller_ip_str << "\ncontroller_port = " << g.controller_port
      << "\n\n[backend.dummy]\nbandwidth = " << backend_.dummy.bandwidth
      << "\nprocess_packets = " << (backend_.dummy.process_packets ? "true" : "false")
      << "\nfail_worker_thread = " << backend_.dummy.fail_worker_thread
      << "\nstall_worker_thread = " << backend_.dummy.stall_worker_thread
      << "\nstall_ms = " << backend_.dummy.stall_ms
      << "\n\n[backend.hip]\ndevice = " << backend_.hip.device << "\nmode = " << backend_.hip.mode
      << "\npacket_ring = " << backend_.hip.packet_ring
      << "\nburst_server = " << (backend_.hip.burst_server ? "true" : "false")
      << "\nbatch_jobs = " << backend_.hip.batch_jobs
      << "\ncoalesce_us = " << backend_.hip.coalesce_us
      << "\nvcl = " << (backend_.hip.vcl ? "true" : "false")
      << "\n\n[backend.xgmi]\nsession = " << backend_.xgmi.session
      << "\nmax_slice_numel = " << backend_.xgmi.max_slice_numel << "\ntimeout_ms = " << backend_.xgmi.timeout_ms
      << "\npush = " << (backend_.xgmi.push ? "true" : "false")
      << "\nfail_setup = " << (backend_.xgmi.fail_setup ? "true" : "false")
      << "\n";
    return o.str();
}

void Config::PrintConfig() const { fprintf(stderr, "[switchml] configuration:\n%s", ToString().c_str()); }

}  // namespace switchml
