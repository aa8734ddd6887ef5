"""GPU parity of the multi-PE path (RS + AG over HIP IPC): 2 and 4 PEs as separate processes on
the one GPU of the test box (the same protocol as one PE per MI355X over xGMI; the 8-GPU run is
the driver's).  Every PE checks its dest against the oracle bit-for-bit (canonical team-order
fold) and against MPICH's MPI_Allreduce golden output (ints / min / max bit-exact; FP sum/prod
within (p-1)*u*sum|x_i| resp. (p-1)*u*|ref|)."""
import multiprocessing as mp
import os
import queue
import sys
import time
import uuid
from pathlib import Path

import pytest

from tests import mp_worker

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.gpu

# The runtime's test hooks (fake device identity, flag memory "unavailable") are compiled into the
# test build only (ishmem_amd/_build.py LIB_TESTHOOKS); the product library refuses them at init.
TESTHOOKS = {"ISHMEM_AMD_LIB": str(ROOT / "ishmem_amd" / "libishmem_amd_testhooks.so")}

# HSA_ENABLE_IPC_MODE_LEGACY is removed from every PE's environment (the box exports it): the
# library's constructor must set it, as for a program launched the reference's way.
ENV = {"ISHMEM_MAX_BLOCKS": 32, "ISHMEM_TIMEOUT_MS": 20000, "ISHMEM_SYMMETRIC_SIZE": "1G",
       "HSA_ENABLE_IPC_MODE_LEGACY": None}


def run_pes(npes: int, scenarios: list[str], timeout: float = 240.0, env: dict | None = None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = f"t{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=mp_worker.run, args=(pe, npes, key, scenarios, q, {**ENV, **(env or {})}))
             for pe in range(npes)]
    for p in procs:
        p.start()
    results = {}
    t0 = time.monotonic()
    try:
        while len(results) < npes:
            # Heartbeat on stderr (run pytest with -s on the GPU box): a long multi-PE case stays
            # visibly alive, and a PE that never reports ends the test at `timeout`.
            try:
                pe, fails = q.get(timeout=min(30.0, max(1.0, timeout - (time.monotonic() - t0))))
            except queue.Empty:
                if time.monotonic() - t0 >= timeout:
                    break
                print(f"[run_pes {npes} PEs {scenarios}] {time.monotonic() - t0:.0f} s, "
                      f"{len(results)} reported", file=sys.stderr, flush=True)
                continue
            results[pe] = fails
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    assert len(results) == npes, f"only {len(results)} of {npes} PEs reported"
    allfails = [f for pe in sorted(results) for f in results[pe]]
    assert not allfails, "\n".join(allfails[:20])


# ll=on: payloads <= 64 KiB take the one-hop granule path; cap: the default, up to the team's
# ring capacity (1 MiB / team size: 512 KiB at 2 PEs, 349,520 B at 3, 256 KiB at 4); off: reduce-
# scatter + all-gather for the same inputs.
LL_ENV = {"on": 65536, "cap": None, "off": 0}


@pytest.mark.parametrize("npes", [2, 4])
@pytest.mark.parametrize("ll", ["on", "cap", "off"])
def test_all_ops_types_vs_oracle_and_mpich_golden(npes, ll):
    run_pes(npes, ["golden"], env={"ISHMEM_LL_MAX_BYTES": LL_ENV[ll]})


@pytest.mark.parametrize("npes", [2, 3])
@pytest.mark.parametrize("ll", ["on", "cap", "off"])
def test_inplace_offsets_edges(npes, ll):
    # offsets_large at 2 and 3 PEs: 70,001 floats (280 KB) and 262,147 bytes take the granule path
    # only with ll=cap, from sources on another phase than dest, guard bytes checked.
    run_pes(npes, ["inplace", "offsets", "offsets_large", "edge"], env={"ISHMEM_LL_MAX_BYTES": LL_ENV[ll]})


def test_stream_staged_team():
    run_pes(4, ["stream", "streams", "staged", "team"])


def test_large_f32_sum_256MiB_per_pe():
    run_pes(2, ["large"], env={"ISHMEM_MAX_BLOCKS": 64})


def test_huge_2p5GiB_per_pe_head_tail_and_2GiB_boundary():
    run_pes(2, ["huge"], env={"ISHMEM_MAX_BLOCKS": 64, "ISHMEM_SYMMETRIC_SIZE": "6G"}, timeout=400)


@pytest.mark.parametrize("npes", [2, 3, 4])
def test_blocking_calls_return_with_dest_final_for_any_stream(npes):
    # The blocking calls' host wait (a stream-written completion word, no hipStreamSynchronize):
    # dest read at once through a non-blocking stream, every kind of blocking collective.
    run_pes(npes, ["blockread"], timeout=200)


@pytest.mark.parametrize("npes", [2, 3, 4, 8])
def test_granule_collectives_chained_without_sync(npes):
    # 32 granule-path reduces / fcollects / scans back to back on one stream, random sizes up to
    # the threshold, random host delays per PE: the rings' parity alternation across modes.
    run_pes(npes, ["llchain"], timeout=200)


@pytest.mark.parametrize("npes", [2, 3, 4])
@pytest.mark.parametrize("ll", ["cap", "off"])
def test_fcollect_collect_scan_vs_tester_patterns_and_oracle(npes, ll):
    # Small staging region so the scan's segment loop runs several times.  ll=cap (the default):
    # fcollect and scans up to the granule ring's capacity take the granule exchange (kLLCollect /
    # kLLInscan / kLLExscan); off: the handshake kernels for every size.
    run_pes(npes, ["collect", "scan"], env={"ISHMEM_STAGING_SIZE": "4M", "ISHMEM_LL_MAX_BYTES": LL_ENV[ll]}, timeout=300)


@pytest.mark.parametrize("npes", [2, 3])
def test_scan_collect_on_the_phased_paths(npes):
    # The threshold forced to 0: at 2 PEs disjoint scans take the direct fold (no scratch), in-place
    # ones and every scan at 3 PEs the phased segments; fcollect / collect the phased pull grid.
    # Tester patterns and seeded inputs vs the oracle, as in the default-path test above.
    run_pes(npes, ["collect", "scan"], env={"ISHMEM_STAGING_SIZE": "4M", "ISHMEM_PHASED_MIN_BYTES": 0,
                                            "ISHMEM_LL_MAX_BYTES": 0}, timeout=300)


def test_launch_parameters_agreed_at_init():
    # Per-PE environments that disagree on the grid cap, the LL threshold and the staging size:
    # init takes the minimum, so the collectives still pair up (a mismatch would otherwise split
    # LL from RS/AG or pair different grids and time out).
    run_pes(3, ["inplace", "offsets", "staged"],
            env={"ISHMEM_MAX_BLOCKS": [32, 8, 64], "ISHMEM_LL_MAX_BYTES": [65536, 0, 4096],
                 "ISHMEM_STAGING_SIZE": ["4M", "8M", "2M"]})


@pytest.mark.parametrize("case", ["p2_default", "p8_default", "p8_one_pe_explicit", "p3_one_pe_off"])
def test_phased_threshold_agreed_at_init(case):
    # Every PE must take the same path (the phased path's barriers are separate launches): the
    # threshold is the maximum over the PEs; by default 4 MiB whatever the topology (round 3
    # turned it off when more than 4 PEs shared a GPU; round 4 runs co-located PEs on the node's
    # path); -1 on any PE disables it.
    npes, env, want = {
        "p2_default": (2, {}, 4 << 20),
        "p8_default": (8, {}, 4 << 20),
        "p8_one_pe_explicit": (8, {"ISHMEM_PHASED_MIN_BYTES": ["64M"] + [""] * 7}, 64 << 20),  # K / M / G suffixes
        "p3_one_pe_off": (3, {"ISHMEM_PHASED_MIN_BYTES": ["", "-1", ""]}, -1),
    }[case]
    env = {"ISHMEM_PHASED_MIN_BYTES": "", **env}  # unset unless the case sets it (an outer setting would leak in)
    run_pes(npes, ["phasedparam", "edge"], env={**env, "PHASED_WANT": want, "ISHMEM_MAX_BLOCKS": 8}, timeout=200)


def test_missing_member_times_out_with_error_instead_of_hanging():
    run_pes(2, ["timeout"], timeout=120)


@pytest.mark.parametrize("npes", [2, 4])
def test_hip_graph_capture_and_replay(npes):
    run_pes(npes, ["graph"])


@pytest.mark.parametrize("ll", ["on", "off"])
def test_eight_pes_compile_time_team_size(ll):
    # p = 8 is the 8 x MI355X node's team size: the register-staged rs_tile<P=8> fold and 8-way
    # LL rings, with 8 processes on the one GPU (small grids so all eight kernels stay resident).
    run_pes(8, ["golden", "inplace", "offsets", "edge", "large", "graph"],
            env={"ISHMEM_MAX_BLOCKS": 8, "ISHMEM_LL_MAX_BYTES": 65536 if ll == "on" else 0},
            timeout=400)


def test_eight_pes_collect_scan_team():
    # The P=8 scan kernel, 8-member fcollect / collect, strided and 2-D teams of an 8-PE world.
    run_pes(8, ["collect", "scan", "team"], env={"ISHMEM_MAX_BLOCKS": 8, "ISHMEM_STAGING_SIZE": "4M"},
            timeout=400)


@pytest.mark.parametrize("direct", ["on", "off"])
def test_two_pe_whole_array_fold(direct):
    # Two members, disjoint buffers, no granule path, phased threshold off: every reduce up to
    # oneshot_p2 bytes folds the whole array on both members — on (default) barrier + one fold
    # grid + barrier (PhaseArgs::whole), off the persistent kernel's one-shot mode.  Golden inputs,
    # offset sweeps (shifted sources), edges, hipGraph replay, the tripwire.
    scen = ["golden", "offsets", "offsets_large", "edge", "graph", "tripwire"] + (["nodirect"] if direct == "off" else [])
    run_pes(2, scen, env={"ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_PHASED_MIN_BYTES": -1, "ISHMEM_MAX_BLOCKS": 64})


@pytest.mark.parametrize("npes", [2, 3])
@pytest.mark.parametrize("shifted", ["vector", "element"])
def test_persistent_kernel_with_shifted_sources(npes, shifted):
    # Sources on another 16-B phase than dest on the persistent kernel (no granule path, no
    # whole-array fold, no phased path): 16-B items laid out by dest with unaligned source loads
    # (default) or the element-granular instantiation (ar_shifted 0); guard bytes checked.
    scen = ["offsets", "offsets_large", "nodirect"] + (["arshift0"] if shifted == "element" else [])
    run_pes(npes, scen, env={"ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_PHASED_MIN_BYTES": -1, "ISHMEM_MAX_BLOCKS": 64})


def test_two_pe_reduce_scatter_allgather_path():
    # At 2 PEs non-in-place reduces take the one-shot fold (below 16 MiB) or the phased path by
    # default; force the persistent RS + AG kernel (and no LL) for the same golden / offset /
    # large cases.
    run_pes(2, ["golden", "offsets", "large"],
            env={"ISHMEM_ONESHOT_P2_MAX_BYTES": 0, "ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_MAX_BLOCKS": 64,
                 "ISHMEM_PHASED_MIN_BYTES": -1})


@pytest.mark.parametrize("npes", [2, 3, 4, 8])
def test_phased_reduce_scatter_allgather_path(npes):
    # The phased path (barrier, one-shot reduce-scatter grid, barrier, one-shot all-gather grid,
    # barrier) forced for every heap reduce with a 16-B body — no LL, no two-member one-shot fold:
    # the golden inputs (every op / type), in place, the offset sweep (head / tail elements, empty
    # chunks), edge cases, 256 MiB per PE compared in full, hipGraph replay and the chained-
    # producer coherence tripwire.  p = 3 runs the run-time team-size fold.
    run_pes(npes, ["phaseevents", "golden", "inplace", "offsets", "offsets_large", "edge", "large", "graph", "tripwire"],
            env={"ISHMEM_PHASED_MIN_BYTES": 0, "ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_ONESHOT_P2_MAX_BYTES": 0,
                 "ISHMEM_MAX_BLOCKS": 64},
            timeout=400)


@pytest.mark.parametrize("npes", [2, 3, 8])
def test_realigned_reduce_scatter_grid_stride_loop(npes):
    # The phased path forced, sources on other 16-B phases than dest (offsets_large), with the
    # realigned reduce-scatter capped at 3 workgroups: its grid-stride loop, which otherwise runs
    # only past 2^31 items per chunk, makes several passes per workgroup.
    run_pes(npes, ["realigncap", "offsets_large"],
            env={"ISHMEM_PHASED_MIN_BYTES": 0, "ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_ONESHOT_P2_MAX_BYTES": 0},
            timeout=300)


@pytest.mark.parametrize("npes", [2, 4])
def test_phased_path_with_nontemporal_peer_loads(npes):
    # The measurement-only mode the N > 1 bench times over xGMI (ISHMEM_PHASED_PEER_NT /
    # set_param "phased_peer_nt": the phased grids load peers' bytes nontemporal instead of sc0 sc1,
    # relying on the kernel-boundary acquire).  On one GPU it must give the same bytes; whether it
    # stays coherent across devices is what the bench's tripwire_peer_nt leg records on the node.
    run_pes(npes, ["golden", "inplace", "offsets", "offsets_large", "large", "tripwire"],
            env={"ISHMEM_PHASED_MIN_BYTES": 0, "ISHMEM_LL_MAX_BYTES": 0, "ISHMEM_ONESHOT_P2_MAX_BYTES": 0,
                 "ISHMEM_PHASED_PEER_NT": 1, "ISHMEM_MAX_BLOCKS": 64},
            timeout=400)


@pytest.mark.parametrize("npes,scenarios", [(4, ["team", "stream", "streams", "staged"]), (6, ["teams2"])])
def test_phased_paths_on_teams_streams_and_staged_buffers(npes, scenarios):
    # The phased paths forced, on strided / nested / 2-D teams, the reference's negative-stride,
    # translate and shared team tests, on-stream calls with *ret and host / non-heap buffers
    # through the staging pipeline.
    run_pes(npes, scenarios, env={"ISHMEM_PHASED_MIN_BYTES": 0, "ISHMEM_MAX_BLOCKS": 16}, timeout=300)


@pytest.mark.parametrize("npes", [2, 8])
def test_one_pe_per_gpu_configuration_emulated(npes):
    # The 8-GPU node's path choices, rehearsed on the one GPU: every PE reports its own device
    # (ISHMEM_TEST_PCI_BUS), so the device share is 1, while the PEs still share one GPU.  Golden
    # inputs, in place, edges, 256 / 64 MiB in full, hipGraph replay and the tripwire must all hold,
    # with the grid cap lifted (ISHMEM_MAX_BLOCKS 1024).  Round 3 had to cap it at 768 / npes: each
    # PE sized its persistent grid for the whole GPU, and eight such waiting grids on one device
    # timed out in the tripwire (profiles/r03/phased_share/r03zh_*).  Now every waiting launch takes
    # at most 1 / wait_slots of the device (kernels.h, "Waiting footprint"), so eight fit at once.
    # Round 6: the team spans (emulated) GPUs, so its thresholds come from the link-byte model
    # (runtime.cpp path_limits; pathparam checks them against the C-ABI's and the restatement in
    # tests/test_path_limits.py) — the granule threshold differs from the co-located run's.
    from tests.test_path_limits import expected
    env = {**TESTHOOKS, "ISHMEM_TEST_PCI_BUS": [f"fake-bus-{i}" for i in range(npes)], "ISHMEM_MAX_BLOCKS": 1024,
           "ISHMEM_PHASED_MIN_BYTES": "", "PHASED_WANT": 4 << 20, "COLOCATED_WANT": 0,
           "LL_LIMIT_WANT": expected(npes, False)[0]}
    run_pes(npes, ["phasedparam", "pathparam", "golden", "inplace", "edge", "large", "graph", "tripwire"], env=env,
            timeout=400)


@pytest.mark.parametrize("npes", [2, 4])
def test_path_thresholds_of_a_colocated_world(npes):
    # The co-located counterpart of the emulated test above: round 5's measured crossovers.
    from tests.test_path_limits import expected
    run_pes(npes, ["pathparam"], env={"COLOCATED_WANT": 1, "LL_LIMIT_WANT": expected(npes, True)[0]}, timeout=120)


@pytest.mark.parametrize("npes,teams_max", [(2, None), (4, 8)])
def test_teams_max_split_allocates_team_memory(npes, teams_max):
    # ISHMEM_TEAMS_MAX (default 64) sizes the team table; each split allocates
    # and exchanges the new team's flag block and ring.  2 PEs: 61 user teams, the 62nd refused
    # naming the variable, reduces on the last / a middle team / WORLD vs the oracle, destroy and
    # re-split; 4 PEs with ISHMEM_TEAMS_MAX=8: 5 teams.
    env = {"ISHMEM_TEAMS_MAX": teams_max if teams_max else "", "TEAMS_WANT": teams_max or 64}
    run_pes(npes, ["teams61", "team"], env=env, timeout=300)


@pytest.mark.parametrize("npes", [2, 3, 4])
def test_inplace_fold_captured_on_one_pe_eager_on_the_others(npes):
    # PE 0 replays a captured in-place 1 MiB / 512 KiB f32 sum while the others
    # call it eagerly (granule path off, so both sizes take the in-place fold); then the graph and
    # in-place scenarios on the same world.
    run_pes(npes, ["inplacegraph", "inplace", "graph"], env={"ISHMEM_LL_MAX_BYTES": 0}, timeout=240)


@pytest.mark.parametrize("npes", [2, 3])
def test_collectives_with_members_passing_different_dest_kinds(npes):
    # PE 0's dest pinned host (blocking) or plain device memory (on a stream), the
    # others' in the heap — the granule fcollect / broadcast decide alike on every member; and the
    # blocking calls' dest read at once by the host (pinned) or another stream (device memory).
    run_pes(npes, ["mixeddest", "hostread"], timeout=240)


@pytest.mark.parametrize("npes,slots", [(2, 16), (4, 16), (8, 32)])
def test_opposite_order_collectives_of_two_teams_one_pe_per_gpu_emulated(npes, slots):
    # collectives of two teams on two streams, issued in opposite orders on the
    # two halves of the PEs, each PE on its own (emulated) device and no grid cap — LL, persistent
    # (1 / 4 MiB) and phased sizes.  Deadlock-free by construction while the co-located PEs' waiting
    # launches fit the device: 2 per PE here, so 8 co-located PEs need 1/32 each (ISHMEM_WAIT_SLOTS);
    # one PE per GPU (4 hardware queues per process) is covered by the default 16.
    env = {**TESTHOOKS, "ISHMEM_TEST_PCI_BUS": [f"fake-bus-{i}" for i in range(npes)], "ISHMEM_MAX_BLOCKS": 1024,
           "ISHMEM_PHASED_MIN_BYTES": "", "ISHMEM_WAIT_SLOTS": slots}
    run_pes(npes, ["opposite"], env=env, timeout=300)


@pytest.mark.parametrize("path", ["phased", "persistent"])
def test_reduce_completes_while_another_kernel_holds_most_cus(path):
    # Weakness of the round-1 protocol (workgroup b of every PE paired with workgroup b of every
    # peer): a collective whose partner workgroups cannot all be resident.  Now any workgroup may
    # satisfy a start flag and work is grabbed (persistent kernel), or no grid waits at all
    # (phased path: only its one-workgroup barriers do), so the reduce runs on whatever CUs are free.
    env = {"ISHMEM_MAX_BLOCKS": 1024}
    if path == "persistent":
        env["ISHMEM_PHASED_MIN_BYTES"] = -1
    run_pes(2, ["occupied"], env=env, timeout=120)


@pytest.mark.parametrize("npes", [2, 4, 8])
def test_coherence_tripwire_chained_producer_reduce(npes):
    # Producer kernel -> on-stream reduce, dest of step k = source of step k+1, alternating teams,
    # offsets and sizes (LL and RS + AG), full window compared on every PE every iteration.
    run_pes(npes, ["tripwire"], env={"ISHMEM_MAX_BLOCKS": 1024}, timeout=300)


@pytest.mark.parametrize("path", ["phased", "persistent"])
def test_config4_eight_pes_1GiB_f32_sum_full_compare(path):
    # BASELINE configs[3] at its size on the one GPU: 8 PEs x 1 GiB, every word compared.  "phased"
    # sets ISHMEM_PHASED_MIN_BYTES=16M on every PE — the path one PE per GPU takes on the node
    # (rs_phase_kernel<P=8> + ag_phase_kernel; also the default now); "persistent" pins the
    # persistent kernel.
    env = {"ISHMEM_MAX_BLOCKS": 1024, "ISHMEM_SYMMETRIC_SIZE": "3G",
           "ISHMEM_PHASED_MIN_BYTES": "16M" if path == "phased" else -1}
    run_pes(8, ["cfg4"], env=env, timeout=600)


@pytest.mark.parametrize("oneshot", ["default", "rs_ag"])
def test_config3_two_pes_1GiB_f32_sum_full_compare(oneshot):
    # BASELINE configs[2]: 2 PEs x 1 GiB f32 sum, every word compared on both PEs (rotating-winner
    # pattern); the default (phased) path and the persistent reduce-scatter + all-gather kernel.
    env = {"ISHMEM_MAX_BLOCKS": 1024, "ISHMEM_SYMMETRIC_SIZE": "3G"}
    if oneshot == "rs_ag":
        env["ISHMEM_ONESHOT_P2_MAX_BYTES"] = 0
        env["ISHMEM_PHASED_MIN_BYTES"] = -1
    run_pes(2, ["cfg3"], env=env, timeout=400)


def test_config1_two_pes_int32_sum_host_buffers():
    # BASELINE configs[0]: int32 sum over host buffers (pageable and pinned, in place and not),
    # 2 PEs, 1 .. 16 Mi elements, bit-exact vs the oracle.
    run_pes(2, ["cfg1"], env={"ISHMEM_MAX_BLOCKS": 256}, timeout=300)


@pytest.mark.parametrize("npes", [2, 8])
def test_config5_min_max_prod_int32_f64_4KiB_to_4GiB(npes):
    # BASELINE configs[4]: min/max/prod x int32/float64, 4 KiB * 4^k up to 4 GiB per PE, every
    # chunk edge checked (4 GiB src + 4 GiB dest + staging per PE: a 9 GiB heap).
    # ISHMEM_PHASED_MIN_BYTES=16M on every PE: from 16 MiB the node's path (rs_phase_kernel<P> +
    # ag_phase_kernel), up to 4 GiB per PE — past 2^32 bytes of payload per PE.
    run_pes(npes, ["cfg5"], env={"ISHMEM_MAX_BLOCKS": 1024, "ISHMEM_SYMMETRIC_SIZE": "9G",
                                 "ISHMEM_PHASED_MIN_BYTES": "16M", "CFG5_MAX_BYTES": 4 << 30}, timeout=900)


@pytest.mark.parametrize("npes", [2, 3, 4, 8])
def test_randomised_protocol_stress(npes):
    # Random (op, type), lengths 1 .. 4 Mi elements, offsets, in place, teams (world, strided,
    # shifted), per-PE grid caps and an occupying kernel on a random PE, chained on one stream;
    # every window vs the oracle's fold, guard bytes around it untouched, *ret clean.
    # STRESS_ITERS / STRESS_SEED override (longer soak runs).
    run_pes(npes, ["stress"], env={"ISHMEM_SYMMETRIC_SIZE": "1G"},
            timeout=float(os.environ.get("STRESS_TIMEOUT", 400)))


@pytest.mark.parametrize("npes", [2, 3, 6])
def test_reference_team_tests_negative_stride_translate_shared(npes):
    # test/unit/team_negative_stride.cpp (reversed team: fcollect order, FP folds in ITS team
    # order), team_translate.cpp (every-2nd / every-3rd PE teams: my_pe / translate_pe -1 off the
    # team, int sum of the per-team-index pattern) and team_shared.cpp (SHARED sum, leader
    # min-reduce in place, size fcollect, leader-team in-place reduce).  6 PEs: PE 0 in both
    # translate teams, PEs 2 / 4 in one, PE 3 in the other.
    run_pes(npes, ["teams2"], env={"ISHMEM_MAX_BLOCKS": 16}, timeout=300)


@pytest.mark.parametrize("kinds", [[0, 1], [1, 1], [2, 2], [0, 2, 1]])
def test_flag_memory_kinds_agree_and_work(kinds):
    # The flag block's memory kind (uncached / fine-grained / coarse-grained VRAM) is agreed at
    # init: every PE ends on the least capable kind any PE starts from (ISHMEM_FLAGS_KIND per PE),
    # and the collectives (LL, RS + AG, fcollect, scan) work on each kind.
    run_pes(len(kinds), ["flagkind", "inplace", "edge", "stream"],
            env={"ISHMEM_FLAGS_KIND": kinds, "FLAGKIND_WANT": max(kinds)})


def test_more_than_2pow32_elements_uint8_xor():
    # 4.5 GiB of uint8 per PE (> 2^32 elements) from a misaligned start, xor over 2 PEs: windows
    # around the 2^32 element / byte boundary, a chunk aliasing point and the ragged end.
    run_pes(2, ["huge8"], env={"ISHMEM_MAX_BLOCKS": 1024, "ISHMEM_SYMMETRIC_SIZE": "10G"}, timeout=500)


@pytest.mark.parametrize("npes", [4, 8])
def test_concurrent_collectives_of_different_teams_on_different_streams(npes):
    # x-team and y-team reduces of a 2-D split plus a WORLD reduce in flight together on three
    # streams (TP / DP groups), no synchronisation between them; full grids per PE.
    run_pes(npes, ["concurrent"], env={"ISHMEM_MAX_BLOCKS": 1024, "ISHMEM_SYMMETRIC_SIZE": "1G"}, timeout=300)


@pytest.mark.parametrize("npes", [2, 3, 4])
def test_broadcast_setup_surface_and_agreed_paths(npes):
    # Host broadcast (every root, dest kinds, staged root source, teams), the setup surface
    # (threading, info, team config), fcollect / scan with mixed source kinds and a refused call
    # that fails on every member without a launch.
    run_pes(npes, ["setup", "bcast"], env={"ISHMEM_STAGING_SIZE": "4M"})


@pytest.mark.parametrize("forced", [False, True])
def test_coarse_grained_flags_across_devices_refused_at_init(forced):
    env = {**TESTHOOKS, "ISHMEM_TEST_FLAGS_UNAVAILABLE": 1, "ISHMEM_TEST_PCI_BUS": ["fake-bus-0", "fake-bus-1"]}
    if forced:
        env["ISHMEM_FLAGS_KIND"] = 2
    run_pes(2, ["refuse"], env=env, timeout=120)


@pytest.mark.parametrize("npes", [2, 3, 4])
def test_team_churn_split_destroy_memory_stable(npes):
    # Round 6: split / reduce / destroy of random strided teams and nested teams, 120 rounds, every
    # result vs the oracle; the flag footprint returns to the base block and the device's free
    # memory does not drift (each split allocates, exports and maps a team block).
    run_pes(npes, ["teamchurn"], env={"CHURN_ITERS": 120}, timeout=300)
