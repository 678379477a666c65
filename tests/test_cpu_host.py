"""CPU-side checks of the product: the C-ABI library loads and exports every
declared symbol, and the host Position API (same bitboard source as the
kernels) reproduces the reference's golden vectors, strings and errors.
No GPU compute is called here."""

import ctypes
import json
import re

import numpy as np
import pytest

from conftest import PKG, ROOT, gpu_available

import othello_mcts as om
from othello_mcts.synthetic import alphazero_state_dict, net_config_from_state_dict, random_opening_actions


def u(x):
    return int(np.int64(x).view(np.uint64))


def test_abi_exports_every_declared_symbol():
    names = set()
    for h in sorted((ROOT / "include").glob("*.h")):
        names |= set(re.findall(r"\b(oamd_[a-z0-9_]+)\s*\(", h.read_text()))
    assert len(names) > 30
    lib = ctypes.CDLL(str(PKG / "othello_mcts" / "liboamd.so"))
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.oamd_abi_version() == 1


def test_product_header_has_no_tuning_or_debug_entry_points():
    """the product ABI is the reference's surface plus the
    batched / self-play / measurement API; scheduling knobs and diagnostics
    live in othello_mcts_amd_experimental.h."""
    product = (ROOT / "include" / "othello_mcts_amd.h").read_text()
    names = set(re.findall(r"\b(oamd_[a-z0-9_]+)\s*\(", product))
    assert not [n for n in names if n.startswith("oamd_debug_")]
    for n in ("oamd_engine_set_pipeline", "oamd_engine_set_nn_chains", "oamd_engine_set_chain_split",
              "oamd_engine_set_adaptive_extra_rounds", "oamd_engine_set_extra_round_grid"):
        assert n not in names, n


def test_loaded_library_was_built_from_the_sources_on_disk():
    """build.py compiles the source hashes into
    liboamd.so; the loaded library must report the hashes of the sources on
    disk (a stale prebuilt library fails here, in smoke() and in bench.py)."""
    from othello_mcts import provenance

    got = provenance.check_loaded_library()
    assert set(got) == {"resnet", "tree", "all"}
    assert all(len(v) == 16 for v in got.values())
    lib = ctypes.CDLL(str(PKG / "othello_mcts" / "liboamd.so"))
    lib.oamd_source_hash.restype = ctypes.c_char_p
    assert lib.oamd_source_hash(b"all").decode() == got["all"]
    assert lib.oamd_source_hash(b"nope") is None


def test_abi_device_count_without_gpu_is_safe():
    lib = ctypes.CDLL(str(PKG / "othello_mcts" / "liboamd.so"))
    n = ctypes.c_int32(-1)
    assert lib.oamd_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


def test_package_surface_matches_reference():
    # cpp/src/othello_mcts/__init__.py:6 exports these four names
    for name in ("MCTS", "Position", "get_flips", "get_legal_moves"):
        assert hasattr(om, name)
    P = om.Position
    for m in ("initial_position", "player", "player1_discs", "player2_discs", "__getitem__",
              "legal_moves", "is_legal_move", "legal_actions", "apply_move", "apply_pass",
              "apply_action", "is_terminal", "__str__"):
        assert hasattr(P, m), m
    for m in ("reset_position", "position", "search", "visit_counts", "mean_action_values",
              "self_play_data", "apply_action", "history_size", "set_history_size", "torch_device",
              "set_torch_device", "torch_pin_memory", "set_torch_pin_memory", "num_simulations",
              "set_num_simulations", "num_threads", "set_num_threads", "batch_size", "set_batch_size",
              "c_puct_base", "set_c_puct_base", "c_puct_init", "set_c_puct_init", "dirichlet_epsilon",
              "set_dirichlet_epsilon", "dirichlet_alpha", "set_dirichlet_alpha"):
        assert hasattr(om.MCTS, m), m


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure mode")
def test_mcts_without_gpu_fails_loudly():
    with pytest.raises(RuntimeError, match="needs a ROCm GPU"):
        om.MCTS()


@pytest.fixture(scope="module")
def bb(golden_dir):
    d = np.load(golden_dir / "bitboards.npz")
    return {k: d[k] for k in d.files}


def test_host_legal_moves_and_flips(bb):
    for me, opp, legal in zip(bb["rnd_me"], bb["rnd_opp"], bb["rnd_legal"]):
        assert om.get_legal_moves(u(me), u(opp)) == u(legal)
    me, opp = bb["rnd_me"], bb["rnd_opp"]
    for i, sq, fl in zip(bb["fl_index"], bb["fl_square"], bb["fl_flips"]):
        assert om.get_flips(1 << (63 - int(sq)), u(me[i]), u(opp[i])) == u(fl)


def test_host_position_replays_golden_games(bb):
    player, p1, p2, legal = bb["pos_player"], bb["pos_p1"], bb["pos_p2"], bb["pos_legal"]
    children = {}
    for k, par in enumerate(bb["ch_parent"]):
        children.setdefault(int(par), []).append(k)
    # walk each game: position i+1 is a child of position i unless i is terminal
    pos = om.Position.initial_position()
    for i in range(len(player)):
        exp = (int(player[i]), u(p1[i]), u(p2[i]), u(legal[i]))
        assert (pos.player(), pos.player1_discs(), pos.player2_discs(), pos.legal_moves()) == exp
        acts = pos.legal_actions()
        assert acts == [int(bb["ch_action"][k]) for k in children.get(i, [])]
        for k in children.get(i, []):
            c = pos.apply_action(int(bb["ch_action"][k]))
            assert (c.player(), c.player1_discs(), c.player2_discs(), c.legal_moves()) == (
                int(bb["ch_player"][k]), u(bb["ch_p1"][k]), u(bb["ch_p2"][k]), u(bb["ch_legal"][k]))
        if pos.is_terminal():
            pos = om.Position.initial_position()
        elif i + 1 < len(player):
            nxt = (int(player[i + 1]), u(p1[i + 1]), u(p2[i + 1]))
            for a in acts:
                c = pos.apply_action(a)
                if (c.player(), c.player1_discs(), c.player2_discs()) == nxt:
                    pos = c
                    break
            else:
                pytest.fail(f"position {i + 1} is not a child of {i}")


def test_position_strings_and_errors(golden_dir):
    g = json.loads((golden_dir / "strings_errors.json").read_text())
    for rec in g["strings"]:
        p = om.Position.initial_position()
        for a in rec["actions"]:
            p = p.apply_action(a)
        assert (p.player(), f"{p.player1_discs():016x}", f"{p.player2_discs():016x}") == (
            rec["player"], rec["p1"], rec["p2"])
        assert str(p) == rec["text"]
    err = g["errors"]
    p = om.Position.initial_position()

    def check(name, fn):
        e = err[name]
        exc = {"invalid_argument": ValueError, "out_of_range": IndexError}[e["kind"]]
        with pytest.raises(exc) as ei:
            fn()
        assert str(ei.value) == e["message"]

    check("at_-1", lambda: p[-1])
    check("at_64", lambda: p[64])
    check("is_legal_move_64", lambda: p.is_legal_move(64))
    check("apply_action_65", lambda: p.apply_action(65))
    check("apply_action_-1", lambda: p.apply_action(-1))
    check("apply_action_0", lambda: p.apply_action(0))
    check("apply_action_64", lambda: p.apply_action(64))
    check("apply_pass", lambda: p.apply_pass())
    check("apply_move_two_bits", lambda: p.apply_move(3))
    check("apply_move_illegal", lambda: p.apply_move(1 << 63))


def test_synthetic_state_dict_keys_and_config():
    sd = alphazero_state_dict(3, 17, 128, 9, 128)
    assert len(sd) == 153  # 153 keys for 128x10b
    params = sum(v.size for k, v in sd.items() if not k.endswith(("running_mean", "running_var", "num_batches_tracked")))
    assert params == 2_698_315  # SURVEY.md §6 (H=8)
    assert net_config_from_state_dict(sd) == {"in_channels": 17, "num_squares": 64, "num_actions": 65,
                                               "conv_channels": 128, "num_residual_blocks": 9,
                                               "value_head_hidden_channels": 128}
    again = alphazero_state_dict(3, 17, 128, 9, 128)
    assert all(np.array_equal(sd[k], again[k]) for k in sd)


def test_random_openings_are_legal():
    for seed in range(50):
        acts = random_opening_actions(seed, 8, om.Position)
        assert len(acts) <= 8
        p = om.Position.initial_position()
        for a in acts:
            p = p.apply_action(a)


def test_resnet_activation_layout_is_bank_conflict_free():
    """Restates the activation layout of csrc/resnet.hip (pad_row, make_tile_pos,
    kgroup_chunk, row pitch 2C+16) and checks the property the kernel relies on:
    for every 3x3 tap, position tile, board and 32-channel block, the 16 lanes of
    each ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table) read 16 distinct
    16-byte slots of a 256-byte bank row, i.e. no bank conflicts."""
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[lane + 32 for lane in g] for g in groups]

    def pad_row(p):
        return ((p >> 3) + 1) * 10 + (p & 7) + 1

    tile = [[None] * 16 for _ in range(4)]
    for n in range(16):
        k = n if n < 4 else (n - 4 if n < 12 else n - 8)
        r = 2 * k + 1 if (n < 4 or n >= 12) else 2 * k
        ps = [p for p in range(64) if pad_row(p) % 16 == r]
        assert len(ps) == 4
        for m in range(4):
            tile[m][n] = ps[m]
    assert sorted(sum(tile, [])) == list(range(64))  # a partition of the board

    def chunk(kg):
        return ((kg & 1) << 1) | (kg >> 1)

    def stride(C):  # GeoT::BROWS: board stride in rows
        return 104 if 512 // C == 2 else 100

    def conflict_free(C, rows):  # rows[lane & 15] = padded row of the lane's square
        pitch = 2 * C + 16
        for t in range(9):
            shift = (t // 3 - 1) * 10 + (t % 3 - 1)
            for kc in range(C // 32):
                for g in groups:
                    addrs = [(rows[lane & 15] + shift) * pitch + (kc * 4 + chunk(lane >> 4)) * 16 for lane in g]
                    if len({(a // 16) % 16 for a in addrs}) != 16:
                        return False
        return True

    for C in (128, 256):
        for b in range(512 // C):
            for m in range(4):
                assert conflict_free(C, [b * stride(C) + pad_row(tile[m][j]) for j in range(16)])

    # edge-row tiling (edge_tile_row): tile m of position group q is board row
    # y = 4h + m of boards P and P + NPAIR; the kernel's 128-position waves (PW
    # 128) own rows 0-7 of their pair (64-position waves, rows 0-3 / 4-7 of a
    # half, are checked too: the layout serves both). Edge-row boards keep no
    # top / bottom border rows (GeoT::ROW0 = 0, BROWS 84 / 88 so that the
    # boards of a pair sit 8 rows apart mod 16): only reads of board rows 0-7
    # happen (tile 0 at dy = -1 and tile 7 at dy = +1 are left out)
    def edge_stride(C):
        return 88 if 512 // C == 2 else 84

    def edge_tile_row(C, q, m, j):
        npair = 512 // C // 2
        P, h = q % npair, q // npair
        y = 4 * h + m
        r0 = (P * edge_stride(C) + y * 10 + 1) & 15
        oddcol = 1 if (j < 4 or j >= 12) else 0
        b = P if j < 8 else P + npair
        x = 2 * (j & 3) + ((r0 & 1) ^ oddcol)
        return b, y, x, b * edge_stride(C) + y * 10 + x + 1

    def edge_conflict_free(C, rows, y):
        pitch = 2 * C + 16
        for t in range(9):
            dy, dx = t // 3 - 1, t % 3 - 1
            if not 0 <= y + dy <= 7:
                continue  # a border tile: its MFMAs and reads are left out
            for kc in range(C // 32):
                for g in groups:
                    addrs = [(rows[lane & 15] + dy * 10 + dx) * pitch + (kc * 4 + chunk(lane >> 4)) * 16 for lane in g]
                    if len({(a // 16) % 16 for a in addrs}) != 16:
                        return False
        return True

    for C in (128, 256):
        boards = 512 // C
        assert (boards // 2 * edge_stride(C)) % 16 == 8 and edge_stride(C) >= 80
        assert boards * edge_stride(C) * (2 * C + 16) + (4 if C == 256 else 3) * 16384 <= 160 * 1024
        for pw in (64, 128):
            seen = set()
            for q in range(boards * 64 // pw):
                for m in range(pw // 16):
                    sq = [edge_tile_row(C, q, m, j) for j in range(16)]
                    assert edge_conflict_free(C, [r for *_, r in sq], sq[0][1])
                    assert len({y for _, y, _, _ in sq}) == 1
                    seen |= {(b, y, x) for b, y, x, _ in sq}
                    assert sq[0][1] == 4 * (q // (boards // 2)) + m  # ascending rows
                    # one column map for all rows of a wave: the register window
                    # reads row r of the wave as base + r board rows
                    r0 = [edge_tile_row(C, q, 0, j)[3] for j in range(16)]
                    assert [r - 10 * m for *_, r in sq] == r0
                    # every tap a kept tile reads stays inside its own board's rows
                    for t in range(9):
                        dy, dx = t // 3 - 1, t % 3 - 1
                        if 0 <= sq[0][1] + dy <= 7:
                            for b, y, x, r in sq:
                                assert b * edge_stride(C) <= r + dy * 10 + dx < b * edge_stride(C) + 80
            assert seen == {(b, y, x) for b in range(boards) for y in range(8) for x in range(8)}


def test_resnet_wide_order_window_and_skips():
    """The tower order of csrc/resnet.hip (wide_cb, wide_dy,
    wide_new; resnet_kstep): per dx and 32-channel block the K-steps dy = -1,
    0, +1. Every (tap, block) once per layer; 128-position waves own rows 0-7,
    so every wave leaves out tile 0 at dy = -1 (row -1) and tile 7 at dy = +1
    (row 8), the same MFMAs in every wave; the 8-row window (row i = board row
    i - 1, rows 1-8 only) holds every row a K-step reads, each read once per
    block and dx, before its first use."""
    def cb(J):
        return J // 3

    def dy(J):
        return J % 3 - 1

    new = {0: 0xFE, 1: 0x100, 2: 0}
    for nb in (4, 8):
        seq = [(dxi + 3 * (dy(J) + 1), cb(J)) for dxi in range(3) for J in range(3 * nb)]
        assert sorted(seq) == [(t, c) for t in range(9) for c in range(nb)]
        held = {}
        for J in range(3 * nb):
            loaded = {i for i in range(9) if (new[J % 3] >> i) & 1}
            assert not (loaded & held.get(cb(J), set()))
            held.setdefault(cb(J), set()).update(loaded)
            tiles = range(1 if dy(J) < 0 else 0, 7 if dy(J) > 0 else 8)
            need = {m + 1 + dy(J) for m in tiles}
            assert need <= held[cb(J)]
            skipped = set(range(8)) - set(tiles)
            assert all(m + dy(J) in (-1, 8) for m in skipped)  # border rows only
        assert all(h == set(range(1, 9)) for h in held.values())


def test_type_stub_covers_the_reference_surface_and_the_module():
    """The .pyi lists every name the compiled module exports, and every
    function/method of the reference's stub (_othello_mcts_impl.pyi:1-74,
    recorded here as names) with the same parameter names."""
    import ast
    from pathlib import Path

    import othello_mcts._othello_mcts_impl as impl

    stub = Path(impl.__file__).with_name("_othello_mcts_impl.pyi")
    tree = ast.parse(stub.read_text())
    names = {n.name for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef))}
    exported = {k for k in dir(impl) if not k.startswith("__")}
    assert exported <= names, exported - names
    classes = {n.name: n for n in tree.body if isinstance(n, ast.ClassDef)}

    def params(cls, meth):
        for f in classes[cls].body:
            if isinstance(f, ast.FunctionDef) and f.name == meth:
                return [a.arg for a in f.args.posonlyargs + f.args.args]
        raise AssertionError(f"{cls}.{meth} missing from the stub")

    ref_mcts = ["reset_position", "position", "search", "visit_counts", "mean_action_values", "self_play_data",
                "apply_action"] + [p + n for n in ("history_size", "torch_device", "torch_pin_memory",
                                                   "num_simulations", "num_threads", "batch_size", "c_puct_base",
                                                   "c_puct_init", "dirichlet_epsilon", "dirichlet_alpha")
                                   for p in ("", "set_")]
    for m in ref_mcts:
        params("MCTS", m)
        assert hasattr(impl.MCTS, m)
    assert params("MCTS", "__init__")[:11] == ["self", "history_size", "torch_device", "torch_pin_memory",
                                               "num_simulations", "num_threads", "batch_size", "c_puct_base",
                                               "c_puct_init", "dirichlet_epsilon", "dirichlet_alpha"]
    for m in ("initial_position", "player", "player1_discs", "player2_discs", "__getitem__", "legal_moves",
              "legal_actions", "apply_move", "apply_pass", "apply_action", "is_terminal", "__str__"):
        params("Position", m)
        assert hasattr(impl.Position, m)


def test_k_tree_reads_no_written_state_through_the_scalar_cache(tmp_path):
    """k_tree orders each leaf's statistic stores before the next
    descent's loads with a wavefront fence, not a vmcnt(0) drain (tree.hip
    wave_order). That holds for VECTOR loads (a wave's vector memory
    operations reach the cache in order); a load the compiler turned into a
    scalar s_load would go through the scalar cache, which does not see the
    wave's vector stores. build.py compiles tree.hip with
    -amdgpu-scalarize-global-loads=false, so no global load is scalarised;
    the gfx950 ISA of the built kernels confirms it: every s_load of k_tree
    (and of its uncapped twin k_tree_wide)
    reads the kernel arguments (one base register, offsets inside the
    argument segment), and every s_load of k_tree_free (which reloads its
    arguments into other registers) lies inside its argument segment."""
    import importlib.util
    import subprocess

    spec = importlib.util.spec_from_file_location("oamd_build", PKG / "build.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert "-amdgpu-scalarize-global-loads=false" in b.UNITS["tree.hip"]
    llvm = "/opt/rocm/lib/llvm/bin"
    obj = PKG / "build" / "tree.hip.o"
    fat, co = tmp_path / "tree.fatbin", tmp_path / "tree.co"
    subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", str(obj), str(tmp_path / "x.o")],
                   check=True)
    subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", "--no-show-raw-insn", str(co)], check=True,
                         capture_output=True, text=True).stdout
    notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    # the metadata map lists each kernel's keys in order: .kernarg_segment_size
    # comes before .name
    kernarg, size = {}, None
    for ln in notes.splitlines():
        if ".kernarg_segment_size:" in ln:
            size = int(ln.split(":", 1)[1])
        elif ".name:" in ln and size is not None:
            kernarg[ln.split(":", 1)[1].strip()] = size
            size = None
    bodies, cur = {}, None
    for ln in dis.splitlines():
        if ln.endswith(">:"):
            cur = ln.split("<", 1)[1].rstrip(">:")
            bodies[cur] = []
        elif cur:
            bodies[cur].append(ln.strip())
    for key, single_base in (("6k_tree", True), ("11k_tree_wide", True), ("11k_tree_free", False)):
        sym = next(n for n in bodies if n.startswith(f"_ZN4oamd{key}E"))
        body = bodies[sym]
        assert len(body) > 1000, sym
        loads = [ln for ln in body if ln.startswith(("s_load", "s_buffer_load"))]
        assert loads, sym
        bases = {re.search(r",\s*(s\[\d+:\d+\]),", ln).group(1) for ln in loads}
        offsets = [int(ln.split("//")[0].split(",")[-1].strip(), 16) for ln in loads]
        assert max(offsets) < kernarg[sym], (sym, hex(max(offsets)))
        if single_base:
            assert len(bases) == 1, bases
