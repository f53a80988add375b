"""Cross-GPU partial coding: the helper and main proxies of a repair or a merge on different GPUs.

The reference's proxies exchange partial blocks over TCP: a helper proxy computes its cluster's partial
(encode_partial_blocks_for_decoding / _for_encoding) and sends it to the main proxy, which adds the
partials (perform_addition) -- help_repair -> main_repair (handle_repair.cpp:249-384, 589-603) and
help_recal -> main_recal (handle_merge.cpp:159,269,319,453).  With the proxies on the GPUs of one node the
partials travel over xGMI by RCCL point to point (ecg_dist.exchange) and the addition runs inside the
main rank's launch.  Each *_state builds one rank's blocks (synthetic splitmix64 bytes of the owner's
stripes, block-major so that a chunk of one slot is one contiguous region), the programs and a
step() that runs one pipelined batch (ecg_dist.pipelined_ring_repair):
  ring_repair_state    Azure-LRC(12,2,2) local repairs, one helper partition on the previous rank;
  global_ring_state    global-parity repairs, four helper partitions on the next four ranks;
  pc_merge_ring_state  PC(4,1,4,1) stripe merging x = 2, old stripe 1's cluster on the previous rank.
bench.py measures them (workloads lrc-repair-ring / lrc-global-ring / pc-merge-ring and the default
line's ring objects); tests/test_gpu_ring.py checks them against the oracle.
"""
from __future__ import annotations

import torch

import ecg
import ecg_dist as D


AZURE_OPTIMAL_PARTS = [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11], [14, 15, 12, 13]]


def azure_local_split(e, k=12, parts=AZURE_OPTIMAL_PARTS):
    """Azure-LRC(12,2,2) local repair of block e (data or local parity): the 6 survivors of its group and
    their split into [helper set, main set] under the OPTIMAL partition.  A partition
    other than the failed block's sends one partial when it holds more than f = 1 survivors, otherwise
    its blocks go to the main proxy directly (handle_repair.cpp:169-176); the main proxy adds its own
    partial over its partition's survivors + the direct blocks (perform_addition,
    handle_repair.cpp:371-376).  For every local pattern of this code that is two sets of three."""
    gid = e // 6 if e < k else e - 14
    group = list(range(6 * gid, 6 * gid + 6)) + [14 + gid]
    surv = [b for b in group if b != e]
    main_part = next(p for p in parts if e in p)
    mine = [b for b in surv if b in main_part]
    helpers = []
    for p in parts:
        if p is main_part:
            continue
        inside = [b for b in surv if b in p]
        if len(inside) > 1:
            helpers.append(inside)
        else:
            mine += inside
    sets = helpers + ([mine] if mine else [])
    assert len(sets) == 2 and all(len(x) == 3 for x in sets), (e, sets)
    return surv, sets


def ring_repair_state(r, S, B, chunk, self_p2p=False):
    """Set-up of bench.py's lrc-repair-ring on rank r: returns (step, rebuilt, e_main, main_view); step()
    runs one pipelined repair of the rank's S stripes.  tests/test_gpu_ring.py drives the same state.
    self_p2p (one rank over RCCL to itself): the helper's blocks get their own store, so the partials
    really move from the helper's slot to the main proxy's."""
    k, l, g = 12, 2, 2
    n = k + g + l
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=True)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    M = ec.make_encoding_matrix()
    cls_local = [e for e in range(n) if e not in (12, 13)]
    helper_progs, main_progs = [], []
    for e in cls_local:
        surv, sets = azure_local_split(e)
        helper_progs.append((ec.partial_decoding_matrix(sets[0], surv, [e]), sets[0], [n]))
        main_progs.append(([list(ec.partial_decoding_matrix(sets[1], surv, [e])) + [1]], sets[1] + [n], [0]))
    helper_progs, main_progs = ecg.Programs(helper_progs), ecg.Programs(main_progs)

    def make_store(owner):
        st = torch.empty((n + 1, S, B), dtype=torch.uint8, device="cuda")
        ecg.fill_random(st, 0xEC0DE, word_offset=D.data_word_offset(owner * S, n + 1, B))
        view = st.permute(1, 0, 2)  # [S][n + 1][B], stripe stride B, block stride S * B
        ecg.encode_batch(k, g + l, M, view[:, :k], view[:, k:n])
        return st, view

    nxt = (r.rank + 1) % r.world
    main_store, main_view = make_store(r.rank)
    help_store, help_view = (main_store, main_view) if (r.world == 1 and not self_p2p) else make_store(nxt)
    idx = torch.arange(S, device="cuda", dtype=torch.int32)
    prog_main = ((idx + r.rank * S) % len(cls_local)).contiguous()
    prog_help = ((idx + nxt * S) % len(cls_local)).contiguous()
    e_main = torch.tensor(cls_local, device="cuda")[prog_main.long()]
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")
    send, recv = help_store[n], main_store[n]

    def helper(c0, c1):
        ecg.matrix_apply_batch_multi(helper_progs, help_view[c0:c1], help_view[c0:c1], prog_of_stripe=prog_help[c0:c1])

    def main_(c0, c1):
        ecg.matrix_apply_batch_multi(main_progs, main_view[c0:c1], rebuilt[c0:c1], prog_of_stripe=prog_main[c0:c1])

    def step(ev=None):
        if ev:
            ev[0].record()
        D.pipelined_ring_repair(S, chunk, helper, main_, send, recv, r)
        if ev:
            ev[1].record()

    return step, rebuilt, e_main, main_view


AZURE_GLOBAL_HELPERS = [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11]]  # the OPTIMAL partition's data parts


def global_ring_state(r, S, B, chunk, self_p2p=False):
    """Set-up of lrc-global-ring on rank r: Azure-LRC(12,2,2) global-parity repairs with partial decoding
    across GPUs.  Stripe i of rank q (global stripe q * S + i) loses global parity e = 12 + (i + q * S) % 2.
    Its k = 12 survivors are the data blocks, which the OPTIMAL partition puts in four parts of three
    ({0,1,2} ... {9,10,11}); the lost block's own part {14,15,12,13}, the main proxy, holds none of them.
    Each part holds more than f = 1 survivor, so each sends one partial (handle_repair.cpp:169-176): the
    helper at shift d = 1..4 is rank q + d, which computes part d - 1's partial of rank q's stripes
    (encode_partial_blocks_for_decoding over the part, survivors = the 12 data blocks) and sends it to rank
    q; the main proxy adds the four partials (perform_addition, handle_repair.cpp:371-376) in one 4 -> 1
    launch.  Helpers on the same rank as their main proxy (shift a multiple of N) copy in place.  Returns
    (step, rebuilt, e_main, main_view)."""
    k, l, g = 12, 2, 2
    n = k + g + l
    # a global repair: the coordinator clears local_or_column (global partial-decoding matrices)
    cp = ecg.CodingParameters(k=k, l=l, g=g, local_or_column=False)
    ec = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, cp)
    ec.init_coding_parameters(cp)
    M = ec.make_encoding_matrix()
    surv = list(range(k))
    # program e - 12 of part p: the part's 3 coefficients of the lost global parity, written to slot 0
    part_progs = [ecg.Programs([(ec.partial_decoding_matrix(part, surv, [e]), part, [0]) for e in (12, 13)])
                  for part in AZURE_GLOBAL_HELPERS]
    add4 = ecg.Programs([([[1, 1, 1, 1]], [0, 1, 2, 3], [0])])
    stores = {}

    def store(owner):  # the owner's S stripes, block-major [n][S][B] as in ring_repair_state
        if owner not in stores:
            st = torch.empty((n, S, B), dtype=torch.uint8, device="cuda")
            ecg.fill_random(st, 0xEC0DE, word_offset=D.data_word_offset(owner * S, n + 1, B))
            view = st.permute(1, 0, 2)
            ecg.encode_batch(k, g + l, M, view[:, :k], view[:, k:n])
            stores[owner] = (st, view)
        return stores[owner]

    main_store, main_view = store(r.rank)
    idx = torch.arange(S, device="cuda", dtype=torch.int32)
    owners = [(r.rank - d) % r.world for d in range(1, 5)]  # shift d: this rank helps owner q - d
    helper_views = [store(o)[1] for o in owners]
    prog_help = [((idx + o * S) % 2).contiguous() for o in owners]
    e_main = (12 + (idx.long() + r.rank * S) % 2)
    send = torch.empty((4, S, B), dtype=torch.uint8, device="cuda")  # send[d - 1]: partials for owner q - d
    recv = torch.empty((4, S, B), dtype=torch.uint8, device="cuda")  # recv[d - 1]: from helper q + d
    send_v, recv_v = send.permute(1, 0, 2), recv.permute(1, 0, 2)  # [S][4][B]
    rebuilt = torch.empty((S, 1, B), dtype=torch.uint8, device="cuda")

    def helper(c0, c1):
        for d in range(4):
            ecg.matrix_apply_batch_multi(part_progs[d], helper_views[d][c0:c1], send_v[c0:c1, d:d + 1],
                                         prog_of_stripe=prog_help[d][c0:c1])

    def xchg(c0, c1):
        if self_p2p or r.world > 1:
            return D.exchange([(send[d, c0:c1], recv[d, c0:c1], -(d + 1)) for d in range(4)], r)
        recv[:, c0:c1].copy_(send[:, c0:c1])  # one rank, no RCCL: every helper is local
        return D.exchange([], r)

    def main_(c0, c1):
        ecg.matrix_apply_batch_multi(add4, recv_v[c0:c1], rebuilt[c0:c1])

    def step(ev=None):
        if ev:
            ev[0].record()
        D.pipelined_ring_repair(S, chunk, helper, main_, send, recv, r, xchg=xchg)
        if ev:
            ev[1].record()

    return step, rebuilt, e_main, main_view


def pc_bid(row, col):
    """rowcol2bid (pc.cpp:326-340) of PC(4,1,4,1): data (row < 4, col < 4) = 4 row + col; the column
    parities (row 4) = 20 + col."""
    return row * 4 + col if row < 4 else 20 + col


def pc_merge_ring_state(r, S, B, chunk, self_p2p=False):
    """Set-up of pc-merge-ring on rank r: config 4's stripe merging with the two old stripes' clusters on
    neighbouring GPUs.  PC(4,1,4,1), merge x = 2, HORIZONTAL: the merged PC(8,1,4,1)'s row parity `row` is
    the XOR of the row's 4 blocks of old stripe 0 and 4 blocks of old stripe 1 (RS(8,1) rows are all ones;
    main_recal / help_recal, handle_merge.cpp:159,269,319,453).  Merge i of rank q keeps old stripe 0 on
    rank q (the main proxy, which writes the new parities) and old stripe 1 on rank q - 1 (the helper): the
    helper XORs each row's 4 blocks into one partial (help_recal's encode_partial_blocks_for_encoding), the
    5 partials of a merge travel to rank q (5 pairs of one exchange per chunk), and the main rank adds its
    own 4 blocks per row and the received partial in one 5 -> 1 launch per row (perform_addition fused).
    Stores are block-major [blocks][S][B], so each row's partials of a chunk are one contiguous region.
    Returns (step, out, expected): out [S][5][B] gets the new row parities; expected(i0, i1) computes them
    on the GPU from regenerated old stripes, for checking."""
    nb = 25
    gen = lambda owner, half, st: ecg.fill_random(  # noqa: E731 -- old stripe `half` of the owner's merges
        st, 0xEC0DE, word_offset=D.data_word_offset((2 * owner + half) * S, nb, B))
    main = torch.empty((nb + 5, S, B), dtype=torch.uint8, device="cuda")  # + 5 slots for received partials
    gen(r.rank, 0, main[:nb])
    nxt = (r.rank + 1) % r.world
    helper = torch.empty((nb, S, B), dtype=torch.uint8, device="cuda")  # old stripe 1 of rank q + 1's merges
    gen(nxt, 1, helper)
    send = torch.empty((5, S, B), dtype=torch.uint8, device="cuda")
    out = torch.empty((S, 5, B), dtype=torch.uint8, device="cuda")
    main_v, help_v, send_v = main.permute(1, 0, 2), helper.permute(1, 0, 2), send.permute(1, 0, 2)
    # one launch stripe per (merge, row): program `row` over merge i = stripe_of[i * 5 + row]
    help_progs = ecg.Programs([([[1] * 4], [pc_bid(row, c) for c in range(4)], [row]) for row in range(5)])
    main_progs = ecg.Programs([([[1] * 5], [pc_bid(row, c) for c in range(4)] + [nb + row], [row])
                               for row in range(5)])
    prog_of = (torch.arange(5 * S, device="cuda", dtype=torch.int32) % 5).contiguous()
    stripe_of = (torch.arange(5 * S, device="cuda", dtype=torch.int32) // 5).contiguous()
    moves = self_p2p or r.world > 1

    def helper_k(c0, c1):
        ecg.matrix_apply_batch_multi(help_progs, help_v, send_v, prog_of_stripe=prog_of[5 * c0:5 * c1],
                                     stripe_of=stripe_of[5 * c0:5 * c1])

    def xchg(c0, c1):
        pairs = [(send[row, c0:c1], main[nb + row, c0:c1], 1) for row in range(5)]
        if moves:
            return D.exchange(pairs, r)
        for snd, rcv, _ in pairs:  # one rank, no RCCL: the helper is local
            rcv.copy_(snd)
        return D.exchange([], r)

    def main_k(c0, c1):
        ecg.matrix_apply_batch_multi(main_progs, main_v, out, prog_of_stripe=prog_of[5 * c0:5 * c1],
                                     stripe_of=stripe_of[5 * c0:5 * c1])

    def step(ev=None):
        if ev:
            ev[0].record()
        D.pipelined_ring_repair(S, chunk, helper_k, main_k, send, None, r, xchg=xchg)
        if ev:
            ev[1].record()

    def expected(i0, i1):
        """New row parities of this rank's merges [i0, i1): old stripe 1 regenerated here."""
        own1 = torch.empty((nb, S, B), dtype=torch.uint8, device="cuda")
        gen(r.rank, 1, own1)
        want = torch.empty((i1 - i0, 5, B), dtype=torch.uint8, device="cuda")
        for row in range(5):
            x = torch.zeros((i1 - i0, B), dtype=torch.uint8, device="cuda")
            for c in range(4):
                x ^= main[pc_bid(row, c), i0:i1] ^ own1[pc_bid(row, c), i0:i1]
            want[:, row] = x
        del own1
        return want

    return step, out, expected
