// miner_main.cpp -- hm_miner: a native GPU miner process for the UNCHANGED
// reference server.  Usage:  hm_miner <host:port>
//
// It does what cmu440/bitcoin/miner/miner.go does -- join with a Join message
// (joinWithServer, :24-34), then for every Request reply with
// NewResult(hash, nonce) (evalRoutine, :36-68; Result write :60-62) -- but
// over the native LSP client (lsp_client.cpp) and with the scan (:46-59,
// init :48-49) on the GPU through hm_scan.  The `upper := Upper+1` uint64
// wrap (:52) is kept.  A GPU failure ends the process (no CPU fallback), like
// an LSP error ends the reference miner; the server then reassigns the chunk
// (server.go:326-376).
//
// Env: HIPMINER_DEVICES=0,1 (default: all visible), HM_LSP_* (lsp_client.hpp).
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
    if (rc != HM_OK) {
        fprintf(stderr, "hm_miner: GPU init failed: %s\n", hm_strerror(rc));
        return 1;
    }
    std::string err;
    auto conn = hm::LspClient::connect(argv[1], hm::LspParams::from_env(), &err);
    if (!conn) {
        printf("Failed to join with server: %s\n", err.c_str());
        hm_close(gpu);
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
                hm_result out;
                rc = hm_scan(gpu, reinterpret_cast<const uint8_t*>(req.data.data()), req.data.size(),
                             req.lower, end - 1, &out);
                if (rc != HM_OK) {
                    fprintf(stderr, "hm_miner: scan failed: %s\n", hm_strerror(rc));
                    status = 2;
                    break;
                }
                res.hash = out.hash;
                res.nonce = out.nonce;
            }
            if (!conn->write(marshal(res))) break;
        }
    }
    if (status == 0) conn->close();
    conn.reset();
    hm_close(gpu);
    return status;
}
