// _othello_mcts_impl — pybind11 host layer over the C ABI (include/othello_mcts_amd.h).
//
// Mirrors the reference's module of the same name (cpp/src/lib/othello_mcts.cpp:49-151):
// free functions get_legal_moves / get_flips, class Position (checked API, same
// exception types and messages), class MCTS (same constructor keywords and
// defaults, same methods, getters and setters). Everything else is additive:
//   _Engine / _Net     raw handles for the batched multi-game path (othello_mcts.batched)
//   BatchedMCTS        G games searched together on one GPU
// This file is plain C++ (no torch headers): torch objects are handled
// through Python calls, exactly like the reference's Pybind11NeuralNet
// (othello_mcts.cpp:19-45) hands tensors to the Python callable.

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <bitset>
#include <cstdio>
#include <cstring>
#include <memory>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "othello_mcts_amd.h"
#include "othello_mcts_amd_experimental.h"

namespace py = pybind11;
using namespace py::literals;

namespace {

// Error code -> Python exception (std::invalid_argument -> ValueError,
// std::out_of_range -> IndexError in the reference's pybind11 module).
void check(int rc) {
    if (rc == OAMD_OK) return;
    const std::string msg = oamd_last_error();
    if (rc == OAMD_INVALID_ARGUMENT) throw py::value_error(msg);
    if (rc == OAMD_OUT_OF_RANGE) throw py::index_error(msg);
    throw std::runtime_error(msg);
}

// ------------------------------------------------------------------ Position
struct Position {
    oamd_position p{};

    static Position initial_position() {
        Position x;
        oamd_initial_position(&x.p);
        return x;
    }
    int player() const { return p.player; }
    uint64_t player1_discs() const { return p.player1_discs; }
    uint64_t player2_discs() const { return p.player2_discs; }
    uint64_t legal_moves() const { return p.legal_moves; }
    bool is_terminal() const { return p.player == 0; }

    // position.h:274-292
    int at(int index) const {
        if (!(0 <= index && index < 64))
            throw py::index_error("Expected 0 <= index < 64, but got " + std::to_string(index) + ".");
        const uint64_t m = 1ULL << (63 - index);
        if (p.player1_discs & m) return 1;
        if (p.player2_discs & m) return 2;
        return 0;
    }
    // position.h:294-306
    bool is_legal_move(int index) const {
        if (!(0 <= index && index < 64))
            throw py::index_error("Expected 0 <= index < 64, but got " + std::to_string(index) + ".");
        return (p.legal_moves & (1ULL << (63 - index))) != 0;
    }
    // position.h:308-326
    std::vector<int> legal_actions() const {
        std::vector<int> a;
        if (p.player == 0) return a;
        if (p.legal_moves == 0) return {64};
        for (int s = 0; s < 64; ++s)
            if (p.legal_moves & (1ULL << (63 - s))) a.push_back(s);
        return a;
    }
    Position applied(int action) const {
        Position c;
        oamd_host_apply_action(&p, action, &c.p);
        return c;
    }
    // position.h:365-380
    Position apply_move(uint64_t move_mask) const {
        if (__builtin_popcountll(move_mask) != 1)
            throw py::value_error("Expected a single bit in move_mask, but got 0b" +
                                  std::bitset<64>(move_mask).to_string() + ".");
        if ((move_mask & p.legal_moves) == 0)
            throw py::value_error("0b" + std::bitset<64>(move_mask).to_string() + " is not a legal move.");
        return applied(63 - __builtin_ctzll(move_mask));
    }
    // position.h:388-400
    Position apply_pass() const {
        if (p.player == 0) throw py::value_error("Pass is not allowed in a terminal position.");
        if (p.legal_moves != 0) throw py::value_error("Pass is not allowed when there are legal moves.");
        return applied(64);
    }
    // position.h:410-427
    Position apply_action(int action) const {
        if (!(0 <= action && action < 65))
            throw py::index_error("Expected 0 <= action < 65, but got " + std::to_string(action) + ".");
        if (action == 64) return apply_pass();
        if ((p.legal_moves & (1ULL << (63 - action))) == 0)
            throw py::value_error(std::to_string(action) + " is not a legal action.");
        return applied(action);
    }
    // position.h:429-456
    std::string to_string() const {
        std::string r = "  a b c d e f g h\n";
        uint64_t m = 1ULL << 63;
        for (int row = 0; row < 8; ++row) {
            r.push_back((char)('1' + row));
            for (int col = 0; col < 8; ++col) {
                r.push_back(' ');
                if (m & p.player1_discs) r += "●";
                else if (m & p.player2_discs) r += "○";
                else if (m & p.legal_moves) r += "×";
                else r += "·";
                m >>= 1;
            }
            if (row < 7) r.push_back('\n');
        }
        return r;
    }
};

// ------------------------------------------------------------------ raw handles
struct Net {
    oamd_net* h = nullptr;
    oamd_net_desc desc{};
    Net(int device, int in_channels, int conv_channels, int num_residual_blocks, int hidden, int dtype) {
        desc = oamd_net_desc{in_channels, conv_channels, num_residual_blocks, hidden, 64, 65, dtype};
        check(oamd_net_create(device, &desc, &h));
    }
    ~Net() {
        if (h) oamd_net_destroy(h);
    }
    std::vector<std::pair<std::string, int64_t>> state_keys() const {
        int32_t n = 0;
        check(oamd_net_state_size(h, &n));
        std::vector<std::pair<std::string, int64_t>> out;
        for (int i = 0; i < n; ++i) {
            const char* k = nullptr;
            int64_t numel = 0;
            check(oamd_net_state_key(h, i, &k, &numel));
            out.emplace_back(k, numel);
        }
        return out;
    }
    void load_state(const std::vector<py::array_t<float, py::array::c_style | py::array::forcecast>>& ts) {
        std::vector<const float*> ptrs;
        ptrs.reserve(ts.size());
        for (auto& t : ts) ptrs.push_back(t.data());
        check(oamd_net_load_state(h, ptrs.data(), (int32_t)ptrs.size()));
    }
    void forward(uintptr_t feat, int rows, uintptr_t pol, uintptr_t val, uintptr_t stream) {
        check(oamd_net_forward(h, reinterpret_cast<const float*>(feat), rows, reinterpret_cast<float*>(pol),
                               reinterpret_cast<float*>(val), reinterpret_cast<void*>(stream)));
    }
    uintptr_t handle() const { return reinterpret_cast<uintptr_t>(h); }
};

struct Engine {
    oamd_engine* h = nullptr;
    int device = 0;
    Engine(int device_, int num_games, int64_t node_capacity, const oamd_search_config& cfg, uint64_t seed)
        : device(device_) {
        check(oamd_engine_create(device, num_games, node_capacity, &cfg, seed, &h));
    }
    ~Engine() {
        if (h) oamd_engine_destroy(h);
    }
    oamd_search_config config() const {
        oamd_search_config c;
        check(oamd_engine_get_config(h, &c));
        return c;
    }
    void set_config(const oamd_search_config& c) { check(oamd_engine_set_config(h, &c)); }
    // Raise when a game's node pool ran out (its search stopped following the
    // reference: leaves could not be expanded) or a descent hit the depth cap.
    void check_health() const {
        int32_t over = 0, capped = 0;
        check(oamd_engine_status(h, &over, &capped));
        if (over)
            throw std::runtime_error("node pool exhausted in " + std::to_string(over) +
                                     " game(s): leaves could not be expanded, so the search no longer "
                                     "matches the reference; create the engine with a larger node_capacity");
        if (capped)
            throw std::runtime_error("search path exceeded the depth cap (127 plies below the root) in " +
                                     std::to_string(capped) + " game(s)");
    }
};

oamd_search_config make_config(int history_size, int num_simulations, int num_threads, int batch_size,
                               float c_puct_base, float c_puct_init, float eps, float alpha) {
    return oamd_search_config{history_size, num_simulations, num_threads, batch_size,
                              c_puct_base, c_puct_init, eps, alpha};
}

// torch bridge helpers (Python-level calls; no libtorch link)
struct Torch {
    py::module_ torch = py::module_::import("torch");
    py::module_ native = py::module_::import("othello_mcts.native");
    uintptr_t current_stream(int device) {
        return torch.attr("cuda").attr("current_stream")(device).attr("cuda_stream").cast<uintptr_t>();
    }
    static uintptr_t ptr(const py::object& t) { return t.attr("data_ptr")().cast<uintptr_t>(); }
};

int device_count() {
    int32_t n = 0;
    oamd_device_count(&n);
    return n;
}

// Parse the reference's torch_device string; the engine itself always lives
// on a GPU (cuda:k -> k, anything else -> the current torch device).
int engine_device_for(const std::string& torch_device) {
    if (device_count() == 0)
        throw std::runtime_error(
            "othello_mcts (MI355X-native) needs a ROCm GPU: no HIP device is visible. "
            "The search tree and kernels run on the GPU; there is no CPU fallback.");
    if (torch_device.rfind("cuda:", 0) == 0) return std::stoi(torch_device.substr(5));
    py::module_ torch = py::module_::import("torch");
    return torch.attr("cuda").attr("current_device")().cast<int>();
}

// ------------------------------------------------------------------ MCTS
// Reference: cpp/src/include/mcts.h:35-216, cpp/src/lib/mcts.cpp.
class MCTS {
public:
    MCTS(int history_size, std::string torch_device, bool torch_pin_memory, int num_simulations, int num_threads,
         int batch_size, float c_puct_base, float c_puct_init, float dirichlet_epsilon, float dirichlet_alpha,
         int64_t node_capacity, uint64_t seed, bool native_nn, const std::string& nn_dtype)
        : torch_device_(std::move(torch_device)), pin_(torch_pin_memory), native_(native_nn) {
        set_nn_dtype(nn_dtype);
        const oamd_search_config c = make_config(history_size, num_simulations, num_threads, batch_size,
                                                 c_puct_base, c_puct_init, dirichlet_epsilon, dirichlet_alpha);
        device_ = engine_device_for(torch_device_);
        if (seed == 0) {
            py::module_ os = py::module_::import("os");
            py::bytes b = os.attr("urandom")(8);
            std::string s = b;
            std::memcpy(&seed, s.data(), 8);
        }
        // one game owns the whole pool and nodes are not reclaimed during a game
        // (DESIGN.md §5): default 2^23 nodes (512 MB) covers a full game at
        // player.py's 3200 simulations per move (~1.6 M nodes)
        if (node_capacity == 0) node_capacity = kSingleGameNodes;
        engine_ = std::make_unique<Engine>(device_, 1, node_capacity, c, seed);
    }
    static constexpr int64_t kSingleGameNodes = (int64_t)1 << 23;

    void reset_position() {
        check(oamd_engine_reset(engine_->h, 0, next_seed()));
        sync();
    }

    Position position() {
        oamd_root_info info;
        check(oamd_engine_root_info(engine_->h, 0, &info, nullptr, nullptr));
        Position p;
        p.p = info.position;
        return p;
    }

    // mcts.h:220-256 + search_thread.cpp:47-128 (per virtual thread NN calls)
    void search(py::object neural_net) {
        Torch T;
        const uintptr_t stream = T.current_stream(device_);
        check(oamd_engine_set_stream(engine_->h, reinterpret_cast<void*>(stream)));
        const oamd_search_config c = engine_->config();
        if (native_) {
            py::object nat = T.native.attr("resolve")(neural_net, device_, c.history_size, nn_dtype_);
            if (!nat.is_none()) {
                auto* net = reinterpret_cast<oamd_net*>(nat.attr("handle").cast<uintptr_t>());
                check(oamd_engine_search(engine_->h, net, nullptr, nullptr));
                engine_->check_health();
                return;
            }
        }
        const int B = c.batch_size, L = c.num_threads * c.batch_size, C = 1 + 2 * c.history_size;
        py::object dev = T.torch.attr("device")("cuda", device_);
        py::object f32 = T.torch.attr("float32");
        py::tuple shape = py::make_tuple(B, C, 8, 8);
        py::object feat_gpu = T.torch.attr("empty")(shape, "dtype"_a = f32, "device"_a = dev);
        const bool on_gpu = torch_device_.rfind("cuda", 0) == 0;
        py::object feat_arg = feat_gpu;
        if (!on_gpu) {
            feat_arg = T.torch.attr("empty")(shape, "dtype"_a = f32, "device"_a = torch_device_,
                                             "pin_memory"_a = pin_);
        }
        int32_t steps = 0;
        check(oamd_engine_search_begin(engine_->h, &steps));
        std::vector<uint8_t> flags(L);
        for (int s = 0; s < steps; ++s) {
            check(oamd_engine_select(engine_->h));
            check(oamd_engine_leaf_flags(engine_->h, flags.data()));
            for (int k = 0; k < c.num_threads; ++k) {
                bool any = false;
                for (int j = 0; j < B; ++j) any |= flags[k * B + j] != 0;
                if (!any) continue;  // search_thread.cpp:102 — all-terminal batch skips the NN
                check(oamd_engine_features(engine_->h, reinterpret_cast<float*>(T.ptr(feat_gpu)), k * B, B));
                if (!on_gpu) feat_arg.attr("copy_")(feat_gpu);
                py::object out = neural_net(feat_arg);
                // othello_mcts.cpp:41-44: policy (B, 65), value (B,)
                py::object pol = out["policy"].attr("detach")().attr("to")("device"_a = dev, "dtype"_a = f32)
                                     .attr("contiguous")();
                py::object val = out["value"].attr("detach")().attr("to")("device"_a = dev, "dtype"_a = f32)
                                     .attr("contiguous")();
                check(oamd_engine_set_evaluation(engine_->h, reinterpret_cast<const float*>(T.ptr(pol)),
                                                 reinterpret_cast<const float*>(T.ptr(val)), k * B, B));
            }
        }
        // the last round's backups (each earlier round was backed up thread by
        // thread inside the next select, the reference's interleaving)
        check(oamd_engine_backup(engine_->h));
        sync();
        engine_->check_health();
    }

    // mcts.cpp:45-52
    std::vector<int> visit_counts() {
        oamd_root_info info;
        int32_t v[65];
        float q[65];
        check(oamd_engine_root_info(engine_->h, 0, &info, v, q));
        return std::vector<int>(v, v + info.num_children);
    }
    // mcts.cpp:54-61
    std::vector<float> mean_action_values() {
        oamd_root_info info;
        int32_t v[65];
        float q[65];
        check(oamd_engine_root_info(engine_->h, 0, &info, v, q));
        return std::vector<float>(q, q + info.num_children);
    }
    // mcts.cpp:63-112 -> {"features": [8 x (C,8,8)], "policy": [8 x (65,)]} fp32 CPU tensors
    py::dict self_play_data() {
        const int C = 1 + 2 * engine_->config().history_size;
        py::array_t<float> f({8, C, 8, 8});
        py::array_t<float> p({8, 65});
        check(oamd_engine_self_play_data(engine_->h, 0, f.mutable_data(), p.mutable_data()));
        py::module_ torch = py::module_::import("torch");
        py::object ft = torch.attr("from_numpy")(f);
        py::object pt = torch.attr("from_numpy")(p);
        py::list fl, pl;
        for (int t = 0; t < 8; ++t) {
            fl.append(ft[py::int_(t)].attr("clone")());
            pl.append(pt[py::int_(t)].attr("clone")());
        }
        return py::dict("features"_a = fl, "policy"_a = pl);
    }
    // mcts.cpp:114-165
    void apply_action(int action) {
        check(oamd_engine_apply_action(engine_->h, 0, action));
        sync();
    }

    // getters / setters (mcts.h:98-200, mcts.cpp:167-241)
    int history_size() const { return engine_->config().history_size; }
    void set_history_size(int v) { update([&](oamd_search_config& c) { c.history_size = v; }); }
    std::string torch_device() const { return torch_device_; }
    void set_torch_device(const std::string& v) {
        const int d = engine_device_for(v);
        if (d != device_)
            throw py::value_error("the native engine keeps its search tree on cuda:" + std::to_string(device_) +
                                  "; create a new MCTS to move it to another GPU");
        torch_device_ = v;
    }
    bool torch_pin_memory() const { return pin_; }
    void set_torch_pin_memory(bool v) { pin_ = v; }
    int num_simulations() const { return engine_->config().num_simulations; }
    void set_num_simulations(int v) { update([&](oamd_search_config& c) { c.num_simulations = v; }); }
    int num_threads() const { return engine_->config().num_threads; }
    void set_num_threads(int v) { update([&](oamd_search_config& c) { c.num_threads = v; }); }
    int batch_size() const { return engine_->config().batch_size; }
    void set_batch_size(int v) { update([&](oamd_search_config& c) { c.batch_size = v; }); }
    float c_puct_base() const { return engine_->config().c_puct_base; }
    void set_c_puct_base(float v) { update([&](oamd_search_config& c) { c.c_puct_base = v; }); }
    float c_puct_init() const { return engine_->config().c_puct_init; }
    void set_c_puct_init(float v) { update([&](oamd_search_config& c) { c.c_puct_init = v; }); }
    float dirichlet_epsilon() const { return engine_->config().dirichlet_epsilon; }
    void set_dirichlet_epsilon(float v) { update([&](oamd_search_config& c) { c.dirichlet_epsilon = v; }); }
    float dirichlet_alpha() const { return engine_->config().dirichlet_alpha; }
    void set_dirichlet_alpha(float v) { update([&](oamd_search_config& c) { c.dirichlet_alpha = v; }); }

    // additive API
    bool native_nn() const { return native_; }
    void set_native_nn(bool v) { native_ = v; }
    std::string nn_dtype() const { return nn_dtype_; }
    void set_nn_dtype(const std::string& v) {
        if (v != "bf16" && v != "fp16")
            throw std::invalid_argument("Expected nn_dtype in {'bf16', 'fp16'}, but got '" + v + "'.");
        nn_dtype_ = v;
    }
    int device() const { return device_; }
    uint64_t game_key() {
        uint64_t k = 0;
        check(oamd_engine_game_key(engine_->h, 0, &k));
        return k;
    }
    void reset_seed(uint64_t seed) {
        check(oamd_engine_reset(engine_->h, 0, seed));
        sync();
    }
    py::dict root_info() {
        oamd_root_info info;
        check(oamd_engine_root_info(engine_->h, 0, &info, nullptr, nullptr));
        return py::dict("visit_count"_a = info.visit_count, "num_children"_a = info.num_children,
                        "node_count"_a = info.node_count, "overflow"_a = info.overflow);
    }

private:
    template <typename F>
    void update(F f) {
        oamd_search_config c = engine_->config();
        f(c);
        engine_->set_config(c);
    }
    void sync() {
        // root queries synchronise on the engine stream; nothing else to do
    }
    uint64_t next_seed() {
        py::module_ os = py::module_::import("os");
        std::string s = py::bytes(os.attr("urandom")(8));
        uint64_t v;
        std::memcpy(&v, s.data(), 8);
        return v;
    }

    std::string torch_device_;
    bool pin_;
    bool native_ = true;
    std::string nn_dtype_ = "fp16";
    int device_ = 0;
    std::unique_ptr<Engine> engine_;
};

}  // namespace

PYBIND11_MODULE(_othello_mcts_impl, m) {
    m.doc() = "MI355X-native othello_mcts (HIP kernels behind a C ABI)";

    m.def("get_legal_moves", &oamd_host_legal_moves, "player_discs"_a, "opponent_discs"_a);
    m.def("get_flips", &oamd_host_flips, "move_mask"_a, "player_discs"_a, "opponent_discs"_a);
    m.def("device_count", &device_count);
    m.def("abi_version", &oamd_abi_version);
    m.def("source_hash", [](const std::string& family) {
        const char* h = oamd_source_hash(family.c_str());
        if (!h) throw py::value_error("unknown source family: " + family);
        return std::string(h);
    });

    py::class_<Position>(m, "Position")
        .def_static("initial_position", &Position::initial_position)
        .def("player", &Position::player)
        .def("player1_discs", &Position::player1_discs)
        .def("player2_discs", &Position::player2_discs)
        .def("__getitem__", &Position::at)
        .def("legal_moves", &Position::legal_moves)
        .def("is_legal_move", &Position::is_legal_move)
        .def("legal_actions", &Position::legal_actions)
        .def("apply_move", &Position::apply_move)
        .def("apply_pass", &Position::apply_pass)
        .def("apply_action", &Position::apply_action)
        .def("is_terminal", &Position::is_terminal)
        .def("__str__", &Position::to_string)
        .def("next_legal_moves", [](const Position& p) { return p.p.next_legal_moves; })
        .def("__eq__", [](const Position& a, const Position& b) {
            return a.p.player == b.p.player && a.p.player1_discs == b.p.player1_discs &&
                   a.p.player2_discs == b.p.player2_discs && a.p.legal_moves == b.p.legal_moves &&
                   a.p.next_legal_moves == b.p.next_legal_moves;
        })
        .def("__repr__", [](const Position& p) {
            char buf[128];
            std::snprintf(buf, sizeof(buf), "Position(player=%d, player1_discs=0x%016llx, player2_discs=0x%016llx)",
                          p.p.player, (unsigned long long)p.p.player1_discs,
                          (unsigned long long)p.p.player2_discs);
            return std::string(buf);
        });

    py::class_<MCTS>(m, "MCTS")
        .def(py::init<int, std::string, bool, int, int, int, float, float, float, float, int64_t, uint64_t, bool,
                      const std::string&>(),
             "history_size"_a = 4, "torch_device"_a = "cpu", "torch_pin_memory"_a = false,
             "num_simulations"_a = 800, "num_threads"_a = 2, "batch_size"_a = 16, "c_puct_base"_a = 20000.0f,
             "c_puct_init"_a = 2.5f, "dirichlet_epsilon"_a = 0.25f, "dirichlet_alpha"_a = 0.5f,
             "node_capacity"_a = 0, "seed"_a = 0, "native_nn"_a = true, "nn_dtype"_a = "fp16")
        .def("reset_position", &MCTS::reset_position)
        .def("position", &MCTS::position)
        .def("search", &MCTS::search)
        .def("visit_counts", &MCTS::visit_counts)
        .def("mean_action_values", &MCTS::mean_action_values)
        .def("self_play_data", &MCTS::self_play_data)
        .def("apply_action", &MCTS::apply_action)
        .def("history_size", &MCTS::history_size)
        .def("set_history_size", &MCTS::set_history_size)
        .def("torch_device", &MCTS::torch_device)
        .def("set_torch_device", &MCTS::set_torch_device)
        .def("torch_pin_memory", &MCTS::torch_pin_memory)
        .def("set_torch_pin_memory", &MCTS::set_torch_pin_memory)
        .def("num_simulations", &MCTS::num_simulations)
        .def("set_num_simulations", &MCTS::set_num_simulations)
        .def("num_threads", &MCTS::num_threads)
        .def("set_num_threads", &MCTS::set_num_threads)
        .def("batch_size", &MCTS::batch_size)
        .def("set_batch_size", &MCTS::set_batch_size)
        .def("c_puct_base", &MCTS::c_puct_base)
        .def("set_c_puct_base", &MCTS::set_c_puct_base)
        .def("c_puct_init", &MCTS::c_puct_init)
        .def("set_c_puct_init", &MCTS::set_c_puct_init)
        .def("dirichlet_epsilon", &MCTS::dirichlet_epsilon)
        .def("set_dirichlet_epsilon", &MCTS::set_dirichlet_epsilon)
        .def("dirichlet_alpha", &MCTS::dirichlet_alpha)
        .def("set_dirichlet_alpha", &MCTS::set_dirichlet_alpha)
        .def("native_nn", &MCTS::native_nn)
        .def("set_native_nn", &MCTS::set_native_nn)
        .def("nn_dtype", &MCTS::nn_dtype)
        .def("set_nn_dtype", &MCTS::set_nn_dtype)
        .def("device", &MCTS::device)
        .def("game_key", &MCTS::game_key)
        .def("reset_seed", &MCTS::reset_seed)
        .def("root_info", &MCTS::root_info);

    // ---- raw handles for the batched path (othello_mcts/batched.py) ----
    py::class_<oamd_search_config>(m, "SearchConfig")
        .def(py::init(&make_config), "history_size"_a = 8, "num_simulations"_a = 800, "num_threads"_a = 2,
             "batch_size"_a = 16, "c_puct_base"_a = 20000.0f, "c_puct_init"_a = 2.5f, "dirichlet_epsilon"_a = 0.25f,
             "dirichlet_alpha"_a = 0.5f)
        .def_readwrite("history_size", &oamd_search_config::history_size)
        .def_readwrite("num_simulations", &oamd_search_config::num_simulations)
        .def_readwrite("num_threads", &oamd_search_config::num_threads)
        .def_readwrite("batch_size", &oamd_search_config::batch_size)
        .def_readwrite("c_puct_base", &oamd_search_config::c_puct_base)
        .def_readwrite("c_puct_init", &oamd_search_config::c_puct_init)
        .def_readwrite("dirichlet_epsilon", &oamd_search_config::dirichlet_epsilon)
        .def_readwrite("dirichlet_alpha", &oamd_search_config::dirichlet_alpha);

    py::class_<Net>(m, "_Net")
        .def(py::init<int, int, int, int, int, int>(), "device"_a, "in_channels"_a, "conv_channels"_a,
             "num_residual_blocks"_a, "value_head_hidden_channels"_a, "dtype"_a = 0)
        .def("state_keys", &Net::state_keys)
        .def("load_state", &Net::load_state)
        .def("forward", &Net::forward, "features"_a, "rows"_a, "policy"_a, "value"_a, "stream"_a = 0)
        .def_property_readonly("handle", &Net::handle);

    py::class_<Engine>(m, "_Engine")
        .def(py::init<int, int, int64_t, const oamd_search_config&, uint64_t>(), "device"_a, "num_games"_a,
             "node_capacity"_a, "config"_a, "seed"_a)
        .def_readonly("device", &Engine::device)
        .def("config", &Engine::config)
        .def("set_config", &Engine::set_config)
        .def("num_games", [](Engine& e) {
            int32_t n;
            check(oamd_engine_num_games(e.h, &n));
            return n;
        })
        .def("set_stream", [](Engine& e, uintptr_t s) { check(oamd_engine_set_stream(e.h, (void*)s)); })
        .def("reset", [](Engine& e, int game, uint64_t seed) { check(oamd_engine_reset(e.h, game, seed)); })
        .def(
            "search",
            [](Engine& e, uintptr_t net, bool sync) -> py::object {
                if (!sync) {  // enqueue only: no counters, the host does not wait
                    check(oamd_engine_search(e.h, reinterpret_cast<oamd_net*>(net), nullptr, nullptr));
                    return py::none();
                }
                int64_t sims = 0, evals = 0;
                check(oamd_engine_search(e.h, reinterpret_cast<oamd_net*>(net), &sims, &evals));
                return py::make_tuple(sims, evals);
            },
            py::arg("net"), py::arg("sync") = true)
        .def("search_begin",
             [](Engine& e) {
                 int32_t steps = 0;
                 check(oamd_engine_search_begin(e.h, &steps));
                 return steps;
             })
        .def("select", [](Engine& e) { check(oamd_engine_select(e.h)); })
        .def("leaf_flags",
             [](Engine& e) {
                 const oamd_search_config c = e.config();
                 int32_t G;
                 check(oamd_engine_num_games(e.h, &G));
                 py::array_t<uint8_t> a((py::ssize_t)G * c.num_threads * c.batch_size);
                 check(oamd_engine_leaf_flags(e.h, a.mutable_data()));
                 return a;
             })
        .def("features",
             [](Engine& e, uintptr_t out, int row_begin, int rows) {
                 check(oamd_engine_features(e.h, reinterpret_cast<float*>(out), row_begin, rows));
             })
        .def("set_evaluation",
             [](Engine& e, uintptr_t pol, uintptr_t val, int row_begin, int rows) {
                 check(oamd_engine_set_evaluation(e.h, reinterpret_cast<const float*>(pol),
                                                  reinterpret_cast<const float*>(val), row_begin, rows));
             })
        .def("backup", [](Engine& e) { check(oamd_engine_backup(e.h)); })
        .def("status",
             [](Engine& e) {
                 int32_t over = 0, capped = 0;
                 check(oamd_engine_status(e.h, &over, &capped));
                 return py::make_tuple(over, capped);
             })
        .def("check_health", [](Engine& e) { e.check_health(); })
        .def("root_info",
             [](Engine& e, int game) {
                 oamd_root_info info;
                 int32_t v[65];
                 float q[65];
                 check(oamd_engine_root_info(e.h, game, &info, v, q));
                 const int nc = info.num_children;
                 return py::dict("player"_a = info.position.player, "player1_discs"_a = info.position.player1_discs,
                                 "player2_discs"_a = info.position.player2_discs,
                                 "legal_moves"_a = info.position.legal_moves,
                                 "next_legal_moves"_a = info.position.next_legal_moves,
                                 "num_children"_a = nc, "visit_count"_a = info.visit_count,
                                 "overflow"_a = info.overflow, "node_count"_a = info.node_count,
                                 "visit_counts"_a = std::vector<int>(v, v + nc),
                                 "mean_action_values"_a = std::vector<float>(q, q + nc));
             })
        .def("root_stats",
             [](Engine& e, uintptr_t visits, uintptr_t q, uintptr_t info) {
                 check(oamd_engine_root_stats(e.h, reinterpret_cast<int32_t*>(visits), reinterpret_cast<float*>(q),
                                              reinterpret_cast<oamd_root_info*>(info)));
             })
        .def("self_play_data",
             [](Engine& e, int game) {
                 const int C = 1 + 2 * e.config().history_size;
                 py::array_t<float> f({8, C, 8, 8});
                 py::array_t<float> p({8, 65});
                 check(oamd_engine_self_play_data(e.h, game, f.mutable_data(), p.mutable_data()));
                 return py::make_tuple(f, p);
             })
        .def("apply_action", [](Engine& e, int game, int action) { check(oamd_engine_apply_action(e.h, game, action)); })
        .def("apply_actions",
             [](Engine& e, uintptr_t actions) {
                 check(oamd_engine_apply_actions(e.h, reinterpret_cast<const int32_t*>(actions)));
             })
        .def("selfplay_move",
             [](Engine& e, int temperature_moves, float temperature, int opening_moves, bool emit, uintptr_t actions,
                uintptr_t finished, uintptr_t feat, uintptr_t pol) {
                 oamd_selfplay_config c{temperature_moves, temperature, opening_moves, emit ? 1 : 0};
                 check(oamd_engine_selfplay_move(e.h, &c, reinterpret_cast<int32_t*>(actions),
                                                 reinterpret_cast<int32_t*>(finished), reinterpret_cast<float*>(feat),
                                                 reinterpret_cast<float*>(pol)));
             })
        .def("selfplay_steps",
             [](Engine& e, uintptr_t net, int n_moves, int temperature_moves, float temperature, int opening_moves,
                bool emit, bool per_move_outputs, uintptr_t actions, uintptr_t finished, uintptr_t feat, uintptr_t pol) {
                 oamd_selfplay_config c{temperature_moves, temperature, opening_moves, emit ? 1 : 0};
                 check(oamd_engine_selfplay_steps(e.h, reinterpret_cast<oamd_net*>(net), &c, n_moves,
                                                  per_move_outputs ? 1 : 0, reinterpret_cast<int32_t*>(actions),
                                                  reinterpret_cast<int32_t*>(finished), reinterpret_cast<float*>(feat),
                                                  reinterpret_cast<float*>(pol)));
             })
        .def("random_openings",
             [](Engine& e, int max_moves, uint64_t seed) { check(oamd_engine_random_openings(e.h, max_moves, seed)); })
        .def("game_key",
             [](Engine& e, int game) {
                 uint64_t k;
                 check(oamd_engine_game_key(e.h, game, &k));
                 return k;
             })
        .def("enable_timing", [](Engine& e, int every) { check(oamd_engine_enable_timing(e.h, every)); },
             py::arg("every") = 1)
        .def("set_pipeline", [](Engine& e, int groups) { check(oamd_engine_set_pipeline(e.h, groups)); })
        .def("set_nn_batch", [](Engine& e, int rows) { check(oamd_engine_set_nn_batch(e.h, rows)); })
        .def("set_nn_chains", [](Engine& e, int chains) { check(oamd_engine_set_nn_chains(e.h, chains)); })
        .def("set_extra_round_grid",
             [](Engine& e, int workgroups) { check(oamd_engine_set_extra_round_grid(e.h, workgroups)); })
        .def("set_chain_split",
             [](Engine& e, int budget, int cuts) { check(oamd_engine_set_chain_split(e.h, budget, cuts)); })
        .def("set_adaptive_extra_rounds",
             [](Engine& e, bool enable, int min_rounds) {
                 check(oamd_engine_set_adaptive_extra_rounds(e.h, enable ? 1 : 0, min_rounds));
             },
             py::arg("enable") = true, py::arg("min_rounds") = 1)
        .def("round_counts", [](Engine& e) {
            int64_t searches = 0, rounds = 0, finals = 0;
            check(oamd_engine_round_counts(e.h, &searches, &rounds, &finals));
            return py::make_tuple(searches, rounds, finals);
        })
        .def("set_free_running",
             [](Engine& e, bool enable) { check(oamd_engine_set_free_running(e.h, enable ? 1 : 0)); })
        .def("set_exact_interleaving",
             [](Engine& e, bool enable) { check(oamd_engine_set_exact_interleaving(e.h, enable ? 1 : 0)); })
        .def("nn_timing", [](Engine& e) {
            float ms;
            int64_t launches, rows;
            check(oamd_engine_nn_timing(e.h, &ms, &launches, &rows));
            return py::make_tuple(ms, launches, rows);
        })
        .def("nn_busy", [](Engine& e) {
            float ms = 0.0f;
            int64_t launches = 0;
            check(oamd_engine_nn_busy(e.h, &ms, &launches));
            return py::make_tuple(ms, launches);
        })
        .def("work_counters", [](Engine& e) {
            int64_t sims = 0, evals = 0;
            check(oamd_engine_work_counters(e.h, &sims, &evals));
            return py::make_tuple(sims, evals);
        })
        .def("descent_depths", [](Engine& e) {
            int64_t leaves = 0, dsum = 0;
            int32_t dmax = 0;
            check(oamd_engine_descent_depths(e.h, &leaves, &dsum, &dmax));
            return py::make_tuple(leaves, dsum, dmax);
        })
        .def("tree_timing", [](Engine& e) {
            float sel, bk;
            int64_t launches;
            check(oamd_engine_tree_timing(e.h, &sel, &bk, &launches));
            return py::make_tuple(sel, bk, launches);
        })
        .def("tree_work", [](Engine& e) {
            int64_t lv = 0, sc = 0, ex = 0, cr = 0, la = 0;
            check(oamd_engine_tree_work(e.h, &lv, &sc, &ex, &cr, &la));
            return py::make_tuple(lv, sc, ex, cr, la);
        });

    // GPU bitboard kernels over device buffers (data_ptr ints) for parity tests
    m.def("_gpu_legal_moves", [](uintptr_t me, uintptr_t opp, uintptr_t out, int64_t n, uintptr_t stream) {
        check(oamd_get_legal_moves((const uint64_t*)me, (const uint64_t*)opp, (uint64_t*)out, n, (void*)stream));
    });
    m.def("_gpu_flips", [](uintptr_t mv, uintptr_t me, uintptr_t opp, uintptr_t out, int64_t n, uintptr_t stream) {
        check(oamd_get_flips((const uint64_t*)mv, (const uint64_t*)me, (const uint64_t*)opp, (uint64_t*)out, n,
                             (void*)stream));
    });
    m.def("_gpu_apply_action", [](uintptr_t in, uintptr_t actions, uintptr_t out, int64_t n, uintptr_t stream) {
        check(oamd_apply_action((const oamd_position*)in, (const int32_t*)actions, (oamd_position*)out, n,
                                (void*)stream));
    });
}
