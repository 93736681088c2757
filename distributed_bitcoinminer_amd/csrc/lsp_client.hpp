// lsp_client.hpp -- native client of the reference's LSP transport, so a GPU
// miner can join the UNCHANGED Go server.
//
// Wire-compatible with cmu440/lsp (cmu440/ = p1/src/github.com/cmu440/):
//   * messages: JSON of lsp.Message (message.go:20-27), Type Connect=0,
//     Data=1, Ack=2 (:13-17); one UDP datagram each
//   * connect: Connect (SeqNum 0) resent every epoch until Ack(connID, 0);
//     fails after EpochLimit epochs (client_impl.go:67-140, 258-286)
//   * data: SeqNum from 1, Size = len(payload), 16-bit end-around-carry
//     checksum of connID, seqNum, size and the payload's LE 16-bit words,
//     NOT complemented (client_impl.go:183-198, checksum.go:10-47);
//     receiver truncates payloads longer than Size and drops shorter or
//     mismatching ones (:200-213)
//   * sliding window of WindowSize unacked messages, resent every epoch with
//     exponential back-off capped at MaxBackOffInterval (:230-257)
//   * an epoch with nothing received sends a heartbeat Ack(connID, 0); after
//     EpochLimit silent epochs the connection is lost (:258-286)
//   * data is delivered to Read in SeqNum order, each Data acked on receipt
//     (:456-471, 510-550)
#pragma once
#include <stdint.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace hm {

struct LspParams {
    int epoch_limit = 5;      // DefaultEpochLimit (params.go:9)
    int epoch_millis = 2000;  // DefaultEpochMillis
    int window_size = 1;      // DefaultWindowSize
    int max_backoff = 0;      // DefaultMaxBackOffInterval
    static LspParams from_env();  // HM_LSP_EPOCH_LIMIT / _EPOCH_MS / _WINDOW / _MAX_BACKOFF
};

namespace lsp {
enum : int { kConnect = 0, kData = 1, kAck = 2 };
struct Msg {
    int type = 0, conn_id = 0, seq = 0, size = 0;
    uint16_t checksum = 0;
    bool has_payload = false;  // false = JSON null
    std::string payload;
};
uint16_t checksum(int conn_id, int seq, int size, const std::string& payload);
std::string encode(const Msg& m);
bool decode(const std::string& bytes, Msg* m);
// integrity check of a received message (truncates an over-long payload)
bool intact(Msg* m);
}  // namespace lsp

class LspClient {
  public:
    // Connects to host:port; nullptr (and *err) if no Ack within EpochLimit epochs.
    static std::unique_ptr<LspClient> connect(const std::string& hostport, const LspParams& p,
                                              std::string* err);
    ~LspClient();
    int conn_id() const { return conn_id_; }
    // Blocks for the next in-order payload; false once the connection is lost.
    bool read(std::string* payload);
    // Queues a payload; false if the connection is already lost.
    bool write(const std::string& payload);
    // Waits until every written payload is acked (or the connection is lost).
    void close();

  private:
    LspClient() = default;
    void loop();
    void send_raw(const std::string& bytes);
    void pump_window_locked();

    struct Out {
        std::string bytes;
        int back_off = 0, waited = 0;
    };
    int fd_ = -1;
    int conn_id_ = 0;
    LspParams p_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool lost_ = false, stop_ = false;
    std::chrono::steady_clock::time_point last_tx_;  // last datagram sent (any kind)
    int next_seq_ = 1;                 // next SeqNum to assign
    int expected_ = 1;                 // next SeqNum to deliver
    std::map<int, Out> inflight_;      // sent, not yet acked
    std::deque<std::pair<int, std::string>> backlog_;  // waiting for the window
    std::map<int, std::string> pending_;               // received out of order
    std::deque<std::string> ready_;                    // in order, for read()
    std::thread th_;
};

}  // namespace hm
