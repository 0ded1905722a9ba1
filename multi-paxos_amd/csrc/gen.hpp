// gen.hpp — synthetic trace generators (host).
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "mpx.h"

namespace mpx {

struct TraceWriter {
    std::string out;
    void begin(uint32_t N, uint32_t semantics, uint64_t M, const std::vector<mpx_epoch> &epochs);
    void node(const std::vector<std::string> &msgs);
    // one node's stream already concatenated: bytes, offs[count + 1] (offs[0] = 0)
    void node_raw(const std::string &bytes, const std::vector<uint64_t> &offs);
};

void enc_value(std::string &s, uint32_t proposer, uint64_t value_id, bool noop, const std::string &payload);
std::string msg_prepare(uint32_t proposer, uint64_t ballot, const std::vector<std::pair<uint64_t, uint64_t>> &ranges);
std::string msg_prepare_reply(uint32_t acceptor, uint64_t ballot, const std::string &body);
std::string msg_reject(uint64_t max_id);
std::string msg_accept(uint32_t proposer, uint64_t accept, uint64_t ballot, const std::string &body);
std::string msg_accept_reply(uint32_t acceptor, uint64_t ballot, uint64_t accept);
std::string msg_commit(uint32_t committer, uint64_t commit, uint64_t ballot, const std::string &body);
std::string msg_commit_reply(uint32_t learner, uint64_t commit);
std::string msg_p_start(uint64_t ballot);
std::string msg_p_batch(uint64_t batch, const std::string &body);

int gen_clean(const mpx_gen_params &p, std::string &out);
int gen_faulty(const mpx_gen_params &p, std::string &out);
int gen_member(const mpx_gen_params &p, std::string &out);

}  // namespace mpx
