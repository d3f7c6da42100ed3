// rl.hpp — C++ mirror of the reference's Env / Agent traits over the C ABI
// (include/rl.h).  Header-only, RAII; every failing call throws rlamd::Error
// carrying rl_last_error().  Used by the CLI drivers in this directory.
//
//   Env<T,COUNT>   src/env.rs:19-49          -> rlamd::Env   (batched over lanes)
//   Agent<T,COUNT> src/agent.rs:47-164       -> rlamd::Agent (batched over lanes)
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rl.h"

namespace rlamd {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};
inline void check(int rc, const char *call) {
    if (rc != RL_OK) throw Error(rc, std::string(call) + ": " + rl_last_error());
}

// reward_history / episode_length of Agent::train / evaluate (src/agent.rs:66-141)
struct Histories {
    std::vector<double> reward;
    std::vector<double> length;
    std::vector<double> training_error;   // per training step (lane 0; recording mode)
};

class Env {
  public:
    Env(const rl_env_config &cfg, uint32_t n_envs, uint64_t seed, uint64_t lane_offset = 0, int device = 0)
        : n_(n_envs) {
        check(rl_env_create(&cfg, n_envs, seed, lane_offset, device, &h_), "rl_env_create");
    }
    ~Env() { rl_env_destroy(h_); }
    Env(const Env &) = delete;
    Env &operator=(const Env &) = delete;
    // Env::reset (src/env.rs:23)
    std::vector<uint64_t> reset() {
        std::vector<uint64_t> obs(n_);
        check(rl_env_reset(h_, obs.data()), "rl_env_reset");
        return obs;
    }
    // Env::step (src/env.rs:24); returns false (and steps nothing) on EnvNotReady
    bool step(const std::vector<uint32_t> &a, std::vector<uint64_t> &obs, std::vector<double> &r,
              std::vector<uint8_t> &term) {
        obs.resize(n_);
        r.resize(n_);
        term.resize(n_);
        const int rc = rl_env_step(h_, a.data(), obs.data(), r.data(), term.data());
        if (rc == RL_E_NOT_READY) return false;
        check(rc, "rl_env_step");
        return true;
    }
    uint32_t size() const { return n_; }

  private:
    rl_env *h_ = nullptr;
    uint32_t n_;
};

class Agent {
  public:
    explicit Agent(const rl_agent_config &cfg) : cfg_(cfg) { check(rl_agent_create(&cfg, &h_), "rl_agent_create"); }
    ~Agent() { rl_agent_destroy(h_); }
    Agent(const Agent &) = delete;
    Agent &operator=(const Agent &) = delete;

    // Agent::set_future_q_value_func (src/agent.rs:48)
    void set_future_q_value_func(int algo) {
        check(rl_agent_set_future_q_value_func(h_, algo), "rl_agent_set_future_q_value_func");
        cfg_.algo = algo;
    }
    // Agent::set_action_selector (src/agent.rs:50), a fresh selector
    void set_action_selector(int selector) {
        check(rl_agent_set_action_selector(h_, selector, cfg_.eps0, cfg_.eps_decay, cfg_.eps_final,
                                           cfg_.decay_kind, cfg_.ucb_c),
              "rl_agent_set_action_selector");
        cfg_.selector = selector;
    }
    // Agent::reset (one_step_agent.rs:43-46)
    void reset() { check(rl_agent_reset(h_), "rl_agent_reset"); }

    // Agent::train (src/agent.rs:66-118).  Histories: lane 0 when n_lanes == 1,
    // else the per-episode-index mean over lanes; training_error needs recording.
    Histories train(uint64_t n_episodes, uint64_t eval_at, bool training_error, rl_stats *st = nullptr) {
        enable_log(n_episodes + (eval_at ? (n_episodes / eval_at + 1) * cfg_.eval_episodes : 0) + 16);
        if (training_error) check(rl_agent_set_recording(h_, 1), "rl_agent_set_recording");
        rl_stats s{};
        check(rl_agent_train(h_, n_episodes, eval_at, &s), "rl_agent_train");
        if (st) *st = s;
        Histories h;
        collect(h, RL_MODE_TRAIN, n_episodes);
        if (training_error) {
            uint64_t n = 0;
            check(rl_agent_take_records(h_, nullptr, 0, &n), "rl_agent_take_records");
            std::vector<rl_step_record> rec(n);
            check(rl_agent_take_records(h_, rec.data(), n, &n), "rl_agent_take_records");
            check(rl_agent_set_recording(h_, 0), "rl_agent_set_recording");
            for (uint64_t i = 0; i < n; i += cfg_.n_lanes)   // [step][lane]: lane 0
                if (rec[i].kind == 2 && rec[i].mode == RL_MODE_TRAIN) h.training_error.push_back(rec[i].td);
        }
        return h;
    }
    // Agent::evaluate (src/agent.rs:120-141)
    Histories evaluate(uint64_t n_episodes, rl_stats *st = nullptr) {
        enable_log(n_episodes + 16);
        rl_stats s{};
        check(rl_agent_evaluate(h_, n_episodes, &s), "rl_agent_evaluate");
        if (st) *st = s;
        Histories h;
        collect(h, RL_MODE_EVAL, n_episodes);
        return h;
    }
    // every finished episode of the last call, lane by lane (for per-episode outcomes)
    const std::vector<rl_episode_record> &last_episodes() const { return eps_; }
    std::vector<double> q() {
        uint32_t S = 0, A = 0, P = 0;
        check(rl_agent_dims(h_, &S, &A, &P), "rl_agent_dims");
        std::vector<double> out((size_t)S * A * P * (cfg_.group_size == 1 ? cfg_.n_lanes : 1));
        check(rl_agent_get_q(h_, out.data(), out.size()), "rl_agent_get_q");
        return out;
    }
    const rl_agent_config &config() const { return cfg_; }
    rl_agent *handle() { return h_; }

  private:
    void enable_log(uint64_t cap) {
        const uint32_t c = (uint32_t)std::min<uint64_t>(cap, 0xffffffffu);
        if (c > log_cap_) {
            check(rl_agent_set_episode_log(h_, c), "rl_agent_set_episode_log");
            log_cap_ = c;
        }
    }
    void collect(Histories &h, int mode, uint64_t n_per_lane) {
        uint64_t n = 0, lost = 0;
        check(rl_agent_take_episodes(h_, nullptr, 0, &n, &lost), "rl_agent_take_episodes");
        eps_.assign(n, rl_episode_record{});
        check(rl_agent_take_episodes(h_, eps_.data(), n, &n, &lost), "rl_agent_take_episodes");
        if (lost) throw Error(RL_E_STATE, "episode log overflow");
        const uint32_t L = cfg_.n_lanes;
        h.reward.assign(n_per_lane, 0.0);
        h.length.assign(n_per_lane, 0.0);
        std::vector<uint64_t> k(L, 0);
        for (const auto &e : eps_) {
            if (e.mode != mode) continue;
            const uint64_t i = k[e.lane]++;
            if (i >= n_per_lane) continue;
            h.reward[i] += e.reward;
            h.length[i] += e.length;
        }
        if (L > 1)
            for (uint64_t i = 0; i < n_per_lane; ++i) { h.reward[i] /= L; h.length[i] /= L; }
    }
    rl_agent_config cfg_;
    rl_agent *h_ = nullptr;
    uint32_t log_cap_ = 0;
    std::vector<rl_episode_record> eps_;
};

}  // namespace rlamd
