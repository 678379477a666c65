// ORACLE TEST INFRASTRUCTURE — never shipped, never linked into the product.
//
// Golden-vector driver for the reference's header-only game core. It is
// compiled (by oracle/Makefile) directly against the reference headers where
// they lie under /root/reference/cpp/src/include:
//   position.h          (bitboard rules, Position, get_legal_moves/get_flips)
//   transformation.h    (D4 action table, positions_to_features)
//   position_iterator.h (SearchNodePositionIterator — parent-chain history)
//   search_node.h       (SearchNode — STL only)
// None of these need libtorch, so this is the reference's own code running.
// The binary writes plain-text records to stdout; tests/golden/make_golden.py
// turns them into the committed fixtures under tests/golden/.
//
// Commands (argv[1]):
//   games  <n_games> <seed>     random self-play games, every position + every child
//   random <n> <seed>           get_legal_moves / get_flips on random disjoint boards
//   table                       transform_action(a, t) for t<8, a<65
//   features <n_games> <seed>   positions_to_features for random chains, H in {1,3,4,8}
//   strings <n_games> <seed>    Position::to_string() for random positions
//   errors                      exception messages of the *_checked API

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "position.h"
#include "position_iterator.h"
#include "search_node.h"
#include "transformation.h"

namespace {

std::uint64_t g_state = 0;

std::uint64_t splitmix64() {
    std::uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int pick(int n) { return static_cast<int>(splitmix64() % static_cast<std::uint64_t>(n)); }

void print_position(const char *tag, const othello::Position &p) {
    std::printf("%s %d %016llx %016llx %016llx\n", tag, p.player(),
                static_cast<unsigned long long>(p.player1_discs()),
                static_cast<unsigned long long>(p.player2_discs()),
                static_cast<unsigned long long>(p.legal_moves()));
}

void cmd_games(int n_games) {
    for (int g = 0; g < n_games; ++g) {
        othello::Position p = othello::Position::initial_position();
        std::printf("G %d\n", g);
        while (true) {
            print_position("P", p);
            if (p.is_terminal()) break;
            std::uint64_t me = p.player() == 1 ? p.player1_discs() : p.player2_discs();
            std::uint64_t opp = p.player() == 1 ? p.player2_discs() : p.player1_discs();
            std::printf("L %016llx\n", static_cast<unsigned long long>(
                                           othello::get_legal_moves(me, opp)));
            std::vector<int> actions = p.legal_actions();
            for (int a : actions) {
                std::uint64_t flips = 0;
                if (a != 64) flips = othello::get_flips(std::uint64_t(1) << (63 - a), me, opp);
                othello::Position c = p.apply_action(a);
                std::printf("A %d %016llx %d %016llx %016llx %016llx\n", a,
                            static_cast<unsigned long long>(flips), c.player(),
                            static_cast<unsigned long long>(c.player1_discs()),
                            static_cast<unsigned long long>(c.player2_discs()),
                            static_cast<unsigned long long>(c.legal_moves()));
            }
            p = p.apply_action(actions[pick(static_cast<int>(actions.size()))]);
        }
    }
}

void cmd_random(int n) {
    for (int i = 0; i < n; ++i) {
        // Random occupancy density so that both sparse and crowded boards appear.
        int density = 1 + pick(7);
        std::uint64_t occ = 0;
        for (int k = 0; k < density; ++k) occ |= splitmix64();
        if (pick(4) == 0) occ &= splitmix64();
        std::uint64_t split = splitmix64();
        std::uint64_t me = occ & split, opp = occ & ~split;
        std::uint64_t legal = othello::get_legal_moves(me, opp);
        std::printf("R %016llx %016llx %016llx\n", static_cast<unsigned long long>(me),
                    static_cast<unsigned long long>(opp),
                    static_cast<unsigned long long>(legal));
        // Flips for every empty square, legal or not (the function is unchecked).
        std::uint64_t empty = ~occ;
        int k = 0;
        for (int sq = 0; sq < 64 && k < 6; ++sq) {
            std::uint64_t m = std::uint64_t(1) << (63 - sq);
            if (!(empty & m)) continue;
            if (pick(3) != 0 && !(legal & m)) continue;
            std::printf("F %d %016llx\n", sq, static_cast<unsigned long long>(
                                                  othello::get_flips(m, me, opp)));
            ++k;
        }
    }
}

void cmd_table() {
    for (int t = 0; t < 8; ++t) {
        std::printf("T %d", t);
        for (int a = 0; a < 65; ++a) std::printf(" %d", othello::transform_action(a, t));
        std::printf("\n");
    }
}

void cmd_features(int n_games) {
    const int hs[4] = {1, 3, 4, 8};
    for (int g = 0; g < n_games; ++g) {
        // Build a parent chain of SearchNodes exactly as MCTS::apply_action does.
        std::vector<std::unique_ptr<othello::SearchNode>> chain;
        chain.push_back(std::make_unique<othello::SearchNode>(
            othello::Position::initial_position()));
        int plies = pick(70);
        for (int k = 0; k < plies; ++k) {
            const othello::Position &p = chain.back()->position;
            if (p.is_terminal()) break;
            std::vector<int> actions = p.legal_actions();
            othello::Position c = p.apply_action(actions[pick(static_cast<int>(actions.size()))]);
            chain.push_back(std::make_unique<othello::SearchNode>(c, chain.back().get()));
        }
        std::printf("C %d %zu\n", g, chain.size());
        for (auto &node : chain) print_position("P", node->position);
        int h = hs[pick(4)];
        int t = pick(8);
        std::vector<float> buf(static_cast<std::size_t>((1 + 2 * h) * 64), -1.0f);
        othello::positions_to_features(
            othello::SearchNodePositionIterator(chain.back().get()),
            othello::SearchNodePositionIterator::end(), buf.data(), h, t);
        std::printf("X %d %d", h, t);
        for (float v : buf) std::printf(" %d", static_cast<int>(v));
        std::printf("\n");
    }
}

void cmd_strings(int n_games) {
    for (int g = 0; g < n_games; ++g) {
        othello::Position p = othello::Position::initial_position();
        int plies = g == 0 ? 0 : pick(61);
        std::vector<int> seq;
        for (int k = 0; k < plies && !p.is_terminal(); ++k) {
            std::vector<int> actions = p.legal_actions();
            seq.push_back(actions[pick(static_cast<int>(actions.size()))]);
            p = p.apply_action(seq.back());
        }
        print_position("P", p);
        std::printf("Q");
        for (int a : seq) std::printf(" %d", a);
        std::printf("\n");
        std::string s = p.to_string();
        std::printf("S");
        for (unsigned char ch : s) std::printf(" %02x", ch);
        std::printf("\n");
    }
}

template <typename F>
void report(const char *name, F f) {
    try {
        f();
        std::printf("E %s ok\n", name);
    } catch (const std::invalid_argument &e) {
        std::printf("E %s invalid_argument %s\n", name, e.what());
    } catch (const std::out_of_range &e) {
        std::printf("E %s out_of_range %s\n", name, e.what());
    }
}

void cmd_errors() {
    othello::Position p = othello::Position::initial_position();
    report("at_-1", [&] { (void)p.at(-1); });
    report("at_64", [&] { (void)p.at(64); });
    report("is_legal_move_64", [&] { (void)p.is_legal_move_checked(64); });
    report("apply_action_65", [&] { (void)p.apply_action_checked(65); });
    report("apply_action_-1", [&] { (void)p.apply_action_checked(-1); });
    report("apply_action_0", [&] { (void)p.apply_action_checked(0); });
    report("apply_action_64", [&] { (void)p.apply_action_checked(64); });
    report("apply_pass", [&] { (void)p.apply_pass_checked(); });
    report("apply_move_two_bits", [&] { (void)p.apply_move_checked(3); });
    report("apply_move_illegal", [&] { (void)p.apply_move_checked(std::uint64_t(1) << 63); });
}

} // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s games|random|table|features|strings|errors ...\n", argv[0]);
        return 2;
    }
    std::string cmd = argv[1];
    int n = argc > 2 ? std::atoi(argv[2]) : 0;
    g_state = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 0;
    if (cmd == "games") cmd_games(n);
    else if (cmd == "random") cmd_random(n);
    else if (cmd == "table") cmd_table();
    else if (cmd == "features") cmd_features(n);
    else if (cmd == "strings") cmd_strings(n);
    else if (cmd == "errors") cmd_errors();
    else return 2;
    return 0;
}
