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
// Liveness: the reference miner answers every Request.  When
// hm_open finds no usable GPU, or an hm_scan fails, this miner says so on
// stderr and scans on the host instead (hm_scan_cpu, bit-identical), from
// then on: a Result is still written, so the unchanged server never has to
// wait out its 10-s drop timer (params.go:8-13) and reassign the chunk
// (server.go:326-376).  Only a bad HIPMINER_DEVICES list ends the process.
//
// Env: HIPMINER_DEVICES=0,1 (default: all visible), HM_CPU_THREADS (host
// scan threads, default the CPUs of the process's affinity mask), HM_LSP_*
// (lsp_client.hpp).  Test hook: HM_MINER_TEST_FAIL_AFTER=N treats the GPU
// scan of the (N+1)-th Request as failed (HM_ERR_HIP, no hm_scan call), so
// tests can drive the mid-run fallback (tests/test_gpu_miner_lsp.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/hipminer.h"
#include "lsp_client.hpp"
#include "wire.hpp"

namespace {

using hm::wire::BitcoinMsg;

std::string marshal(const BitcoinMsg& m) { return hm::wire::marshal_bitcoin(m); }

BitcoinMsg unmarshal(const std::string& payload) {
    BitcoinMsg m;
    hm::wire::unmarshal_bitcoin(payload, &m);  // error ignored (miner.go:45)
    return m;
}

std::vector<int> devices_from_env() {
    std::vector<int> ds;
    const char* v = getenv("HIPMINER_DEVICES");
    if (!v) return ds;
    std::string s = v;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        const std::string tok = s.substr(i, j - i);
        if (!tok.empty()) ds.push_back(atoi(tok.c_str()));
        i = j + 1;
    }
    return ds;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        printf("Usage: ./%s <hostport>", argv[0]);
        return 0;
    }
    std::vector<int> ds = devices_from_env();
    hm_ctx* gpu = nullptr;
    int rc = hm_open(ds.empty() ? nullptr : ds.data(), (int)ds.size(), &gpu);
    if (rc == HM_ERR_INVALID) {
        fprintf(stderr, "hm_miner: bad HIPMINER_DEVICES: %s\n", hm_strerror(rc));
        return 1;
    }
    const char* th = getenv("HM_CPU_THREADS");
    const int cpu_threads = th ? atoi(th) : 0;
    const char* fa = getenv("HM_MINER_TEST_FAIL_AFTER");
    long gpu_scans_left = fa && *fa ? atol(fa) : -1;  // < 0: no injected failure
    if (rc != HM_OK) {
        gpu = nullptr;
        fprintf(stderr, "hm_miner: NO GPU (%s): every Request is scanned on the host "
                        "(hm_scan_cpu), orders of magnitude slower\n", hm_strerror(rc));
    }
    std::string err;
    auto conn = hm::LspClient::connect(argv[1], hm::LspParams::from_env(), &err);
    if (!conn) {
        printf("Failed to join with server: %s\n", err.c_str());
        if (gpu) hm_close(gpu);
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
                const uint8_t* msg = reinterpret_cast<const uint8_t*>(req.data.data());
                hm_result out;
                rc = HM_ERR_NO_DEVICE;
                if (gpu) {
                    rc = gpu_scans_left == 0
                             ? HM_ERR_HIP
                             : hm_scan(gpu, msg, req.data.size(), req.lower, end - 1, &out);
                    if (gpu_scans_left > 0) --gpu_scans_left;
                    if (rc != HM_OK) {
                        fprintf(stderr, "hm_miner: GPU scan FAILED (%s): this and every later "
                                        "Request are scanned on the host (hm_scan_cpu)\n",
                                hm_strerror(rc));
                        hm_close(gpu);
                        gpu = nullptr;
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
                res.hash = out.hash;
                res.nonce = out.nonce;
            }
            if (!conn->write(marshal(res))) break;
        }
    }
    if (status == 0) conn->close();
    conn.reset();
    if (gpu) hm_close(gpu);
    return status;
}
