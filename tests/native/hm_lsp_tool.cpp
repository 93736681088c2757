// hm_lsp_tool -- host-only test driver of the native LSP client and wire codec
// (test infrastructure; built into build/ by `make -C distributed_bitcoinminer_amd/csrc tools`).
//   hm_lsp_tool echo <host:port>                 join with "hello", echo every payload back
//   hm_lsp_tool checksum <connID> <seq> <hex>    lsp checksum of a payload
//   hm_lsp_tool encode <type> <connID> <seq> <hex|->   lsp.Message JSON
//   hm_lsp_tool decode <json>                    "type connID seq size checksum intact hex"
//   hm_lsp_tool jsonstr <hex>                    Go encoding/json string of bytes
//   hm_lsp_tool bitcoin <json>                   unmarshal then marshal a bitcoin.Message
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../distributed_bitcoinminer_amd/csrc/lsp_client.hpp"
#include "../../distributed_bitcoinminer_amd/csrc/wire.hpp"

static std::string unhex(const char* h) {
    std::string out;
    if (!strcmp(h, "-")) return out;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) {
        char b[3] = {h[i], h[i + 1], 0};
        out.push_back((char)strtol(b, nullptr, 16));
    }
    return out;
}
static std::string tohex(const std::string& s) {
    static const char* x = "0123456789abcdef";
    std::string o;
    for (unsigned char c : s) { o += x[c >> 4]; o += x[c & 15]; }
    return o;
}

int main(int argc, char** argv) {
    if (argc >= 3 && !strcmp(argv[1], "echo")) {
        std::string err;
        auto c = hm::LspClient::connect(argv[2], hm::LspParams::from_env(), &err);
        if (!c) { printf("connect failed: %s\n", err.c_str()); return 3; }
        printf("connected %d\n", c->conn_id());
        fflush(stdout);
        if (!c->write("hello")) return 4;
        std::string p;
        int n = 0;
        while (c->read(&p)) {
            if (p == "quit") break;
            if (!c->write(p)) return 5;
            ++n;
        }
        c->close();
        printf("echoed %d\n", n);
        return 0;
    }
    if (argc >= 5 && !strcmp(argv[1], "checksum")) {
        const std::string p = unhex(argv[4]);
        printf("%u\n", hm::lsp::checksum(atoi(argv[2]), atoi(argv[3]), (int)p.size(), p));
        return 0;
    }
    if (argc >= 6 && !strcmp(argv[1], "encode")) {
        hm::lsp::Msg m;
        m.type = atoi(argv[2]);
        m.conn_id = atoi(argv[3]);
        m.seq = atoi(argv[4]);
        if (strcmp(argv[5], "-")) {
            m.payload = unhex(argv[5]);
            m.has_payload = true;
            m.size = (int)m.payload.size();
            m.checksum = hm::lsp::checksum(m.conn_id, m.seq, m.size, m.payload);
        }
        printf("%s\n", hm::lsp::encode(m).c_str());
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "decode")) {
        hm::lsp::Msg m;
        if (!hm::lsp::decode(argv[2], &m)) { printf("bad\n"); return 0; }
        const bool ok = hm::lsp::intact(&m);
        printf("%d %d %d %d %u %d %s\n", m.type, m.conn_id, m.seq, m.size, m.checksum, ok ? 1 : 0,
               m.has_payload ? tohex(m.payload).c_str() : "null");
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "jsonstr")) {
        printf("%s\n", hm::wire::json_string_go(unhex(argv[2])).c_str());
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "bitcoin")) {
        hm::wire::BitcoinMsg m;
        const bool ok = hm::wire::unmarshal_bitcoin(argv[2], &m);
        printf("%d %s\n", ok ? 1 : 0, hm::wire::marshal_bitcoin(m).c_str());
        return 0;
    }
    fprintf(stderr, "usage: see source\n");
    return 2;
}
