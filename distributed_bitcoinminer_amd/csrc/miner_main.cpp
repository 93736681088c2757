// miner_main.cpp -- hm_miner: a native GPU miner process for the UNCHANGED
// reference server.  Usage:  hm_miner <host:port>
//
// It does what cmu440/bitcoin/miner/miner.go does -- join with a Join message
// (joinWithServer, :24-34), then for every Request reply with
// NewResult(hash, nonce) (evalRoutine, :36-68; Result write :60-62) -- but
// over the native LSP client (lsp_client.cpp) and with the scan (:46-59,
// init :48-49) on the GPU through hm_scan.  The `upper := Upper+1` uint64
// wrap (:52) is kept.
//
// Liveness: the reference miner answers every Request.
//   * No usable GPU at start (no device, a HIPMINER_DEVICES ordinal that is
//     not visible, any hm_open failure): say so on stderr and scan on the host
//     (hm_scan_cpu, bit-identical).
//   * A GPU scan that fails (any rc) or misses its deadline: that Request is
//     answered on the host, the context is closed (an abandoned one without
//     waiting on the device), and the GPU is tried again -- a new hm_open --
//     on a later Request, after a backoff that doubles per failure (1 s .. 60
//     s), so one transient error does not leave this miner, and with it every
//     later job the server splits over all miners, at host speed for good.
//   * Every GPU scan runs under a deadline (HM_OPT_DEADLINE_MS, auto: 2 s + 8x
//     the modelled kernel time).  Without it a hung GPU scan would block this
//     process while the LSP thread keeps heartbeating, and the server, which
//     reassigns only dropped miners (server.go:326-376), would wait forever.
//   * A device fault that aborts the process ends the LSP heartbeats: the
//     server drops the miner after EpochLimit epochs and reassigns its chunk,
//     the reference's own failure path (CS4).
// Only a malformed HIPMINER_DEVICES list ends the process.
//
// Env: HIPMINER_DEVICES=0,1 (default: all visible), HM_SCAN_DEADLINE_MS (ms
// per GPU scan; 0 = none; default auto), HM_MINER_RETRY_MS (first backoff
// before the GPU is retried, default 1000), HM_CPU_THREADS (host scan threads,
// default the CPUs of the process's affinity mask), HM_MINER_VERBOSE=1 (one
// stderr line per Request: range, gpu|host, ms), HM_LSP_* (lsp_client.hpp).
// Test hook: HM_MINER_TEST_FAIL_AFTER=N treats the GPU scan of the (N+1)-th
// Request as failed (HM_ERR_HIP, no hm_scan call), once, so tests can drive
// the mid-run fallback and the GPU's return (tests/test_gpu_miner_lsp.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/hipminer.h"
#include "lsp_client.hpp"
#include "wire.hpp"

namespace {

using hm::wire::BitcoinMsg;
using clk = std::chrono::steady_clock;

std::string marshal(const BitcoinMsg& m) { return hm::wire::marshal_bitcoin(m); }

BitcoinMsg unmarshal(const std::string& payload) {
    BitcoinMsg m;
    hm::wire::unmarshal_bitcoin(payload, &m);  // error ignored (miner.go:45)
    return m;
}

// HIPMINER_DEVICES: comma-separated non-negative ordinals (empty entries
// skipped).  Returns false on a malformed entry -- the one fatal error.
bool devices_from_env(std::vector<int>* ds) {
    const char* v = getenv("HIPMINER_DEVICES");
    if (!v) return true;
    const std::string s = v;
    size_t i = 0;
    while (i <= s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        std::string tok = s.substr(i, j - i);
        tok.erase(0, tok.find_first_not_of(" \t"));
        tok.erase(tok.find_last_not_of(" \t") + 1);
        if (!tok.empty()) {
            char* end = nullptr;
            const long n = strtol(tok.c_str(), &end, 10);
            if (*end != '\0' || n < 0 || n > 1 << 20) return false;
            ds->push_back((int)n);
        }
        i = j + 1;
    }
    return true;
}

long env_long(const char* name, long dflt) {
    const char* v = getenv(name);
    return v && *v ? atol(v) : dflt;
}

// The GPU side of the miner: a context when one is open, else the time the
// next hm_open may be tried.
struct Gpu {
    std::vector<int> devices;
    long deadline_ms;  // HM_OPT_DEADLINE_MS value (-1 = auto)
    long retry_ms;     // current backoff
    hm_ctx* ctx = nullptr;
    clk::time_point retry_at{};
    bool abandoned_any = false;  // some context timed out: skip runtime teardown at exit

    int open() {
        hm_ctx* c = nullptr;
        int rc = hm_open(devices.empty() ? nullptr : devices.data(), (int)devices.size(), &c);
        if (rc == HM_OK && deadline_ms != 0) rc = hm_set_option(c, HM_OPT_DEADLINE_MS, deadline_ms);
        if (rc != HM_OK) {
            if (c) hm_close(c);
            return rc;
        }
        ctx = c;
        return HM_OK;
    }
    // after a failed open or scan: no context until the backoff has passed
    void back_off() {
        retry_at = clk::now() + std::chrono::milliseconds(retry_ms);
        retry_ms = std::min(std::max(2 * retry_ms, 1000L), 60000L);
    }
    void drop(int rc) {
        if (rc == HM_ERR_TIMEOUT) abandoned_any = true;
        hm_close(ctx);  // an abandoned context: host memory only, no device wait
        ctx = nullptr;
        back_off();
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        printf("Usage: ./%s <hostport>", argv[0]);
        return 0;
    }
    Gpu gpu;
    if (!devices_from_env(&gpu.devices)) {
        fprintf(stderr, "hm_miner: bad HIPMINER_DEVICES=%s (comma-separated ordinals)\n",
                getenv("HIPMINER_DEVICES"));
        return 1;
    }
    gpu.deadline_ms = env_long("HM_SCAN_DEADLINE_MS", -1);
    gpu.retry_ms = std::max(0L, env_long("HM_MINER_RETRY_MS", 1000));
    const int cpu_threads = (int)env_long("HM_CPU_THREADS", 0);
    const bool verbose = env_long("HM_MINER_VERBOSE", 0) != 0;
    long gpu_scans_left = env_long("HM_MINER_TEST_FAIL_AFTER", -1);  // < 0: no injected failure
    int rc = gpu.open();
    if (rc != HM_OK) {
        fprintf(stderr, "hm_miner: NO GPU (%s): Requests are scanned on the host "
                        "(hm_scan_cpu), orders of magnitude slower; hm_open is retried "
                        "with backoff\n", hm_strerror(rc));
        gpu.back_off();
    }
    std::string err;
    auto conn = hm::LspClient::connect(argv[1], hm::LspParams::from_env(), &err);
    if (!conn) {
        printf("Failed to join with server: %s\n", err.c_str());
        if (gpu.ctx) hm_close(gpu.ctx);
        return 0;
    }
    BitcoinMsg join;  // NewJoin (message.go:47-49)
    int status = 0;
    if (conn->write(marshal(join))) {
        std::string payload;
        while (conn->read(&payload)) {
            const BitcoinMsg req = unmarshal(payload);
            BitcoinMsg res;
            res.type = 2;  // Result
            res.hash = ~0ull;
            res.nonce = 0;  // miner.go:48-49
            const uint64_t end = req.upper + 1;  // miner.go:52, wraps
            if (req.lower < end) {
                const auto t0 = clk::now();
                const uint8_t* msg = reinterpret_cast<const uint8_t*>(req.data.data());
                hm_result out;
                if (!gpu.ctx && clk::now() >= gpu.retry_at) {
                    rc = gpu.open();
                    if (rc == HM_OK) fprintf(stderr, "hm_miner: GPU (re)opened\n");
                    else gpu.back_off();
                }
                rc = HM_ERR_NO_DEVICE;
                const char* where = "host";
                if (gpu.ctx) {
                    if (gpu_scans_left == 0) {
                        rc = HM_ERR_HIP;  // test hook: one injected failure
                        gpu_scans_left = -1;
                    } else {
                        rc = hm_scan(gpu.ctx, msg, req.data.size(), req.lower, end - 1, &out);
                        if (gpu_scans_left > 0) --gpu_scans_left;
                    }
                    if (rc == HM_OK) {
                        where = "gpu";
                    } else {
                        fprintf(stderr, "hm_miner: GPU scan FAILED (%s): this Request is scanned "
                                        "on the host (hm_scan_cpu); the GPU is retried in %ld ms\n",
                                hm_strerror(rc), gpu.retry_ms);
                        gpu.drop(rc);
                    }
                }
                if (rc != HM_OK) {
                    rc = hm_scan_cpu(msg, req.data.size(), req.lower, end - 1, cpu_threads, &out);
                    if (rc != HM_OK) {
                        fprintf(stderr, "hm_miner: host scan failed: %s\n", hm_strerror(rc));
                        status = 2;
                        break;
                    }
                }
                if (verbose)
                    fprintf(stderr, "hm_miner: Request [%llu, %llu] on %s in %.3f ms\n",
                            (unsigned long long)req.lower, (unsigned long long)(end - 1), where,
                            std::chrono::duration<double, std::milli>(clk::now() - t0).count());
                res.hash = out.hash;
                res.nonce = out.nonce;
            }
            if (!conn->write(marshal(res))) break;
        }
    }
    if (status == 0) conn->close();
    conn.reset();
    if (gpu.ctx) hm_close(gpu.ctx);
    if (gpu.abandoned_any) {
        // a timed-out scan may still occupy the GPU: leave without the HIP
        // runtime's teardown, which could wait on it
        fflush(stdout);
        fflush(stderr);
        _exit(status);
    }
    return status;
}
