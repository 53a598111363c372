"""Pin the oracle's rate limiter (internal/server/rate.go, the inMemory size
hooks in inmemory.go:139-246 and the raft.go hooks 551-621, 660-683, 989-1008,
1779-1785) with the reference's own tests: rate_test.go, the TestRateLimit*
cases of inmemory_test.go:558-660 and raft_test.go:2783-2898.

testRateLimit (raft_etcd_test.go:44) is settings.LargeEntitySize * 4 =
256 MiB; the raft cases here use 64 KiB with a Cmd one byte over it (the
limiter only compares sizes, so the outcome is the same and the test stays
light)."""
import pytest

import oracle as O
from test_oracle_inmem import InMem

U64_MAX = (1 << 64) - 1
TEST_RATE_LIMIT = 64 * 1024
ENTRY_IN_MEM = 80  # unsafe.Sizeof(pb.Entry) on 64-bit Go (raftpb/raft.go:316)


def _rl(max_size):
    """A raft whose limiter is server.NewRateLimiter(max_size): the rate.go
    unit cases drive it directly."""
    r = O.Raft.new(1, [1])
    r.rl_set_max(max_size)
    return r


def in_mem_size(cmd_lens):
    """GetEntrySliceInMemSize (raftpb/raft.go:311-322)."""
    return sum(n + ENTRY_IN_MEM for n in cmd_lens)


# ------------------------------------------------------------ rate_test.go
@pytest.mark.parametrize("max_size,enabled", [(0, False), (U64_MAX, False), (1, True),
                                              (U64_MAX - 1, True)])
def test_rate_limiter_can_be_enabled(max_size, enabled):  # rate_test.go:22-38
    assert bool(_rl(max_size).rl_enabled()) == enabled


def test_in_mem_log_size_is_accessible():  # rate_test.go:40-57
    r = _rl(100)
    assert r.rl_get() == 0
    r.rl_increase(100)
    assert r.rl_get() == 100
    r.rl_decrease(10)
    assert r.rl_get() == 90
    r.rl_set(243)
    assert r.rl_get() == 243


def test_rate_limiter_tick():  # rate_test.go:59-67
    r = _rl(100)
    for i in range(100):
        r.rl_heartbeat_tick()
        assert r.rl_tick() == i + 1


def test_follower_state_can_be_set():  # rate_test.go:69-100
    r = _rl(100)
    r.rl_set_follower(100, 1)
    r.rl_set_follower(101, 2)
    r.rl_heartbeat_tick()
    r.rl_heartbeat_tick()
    r.rl_set_follower(101, 4)
    r.rl_set_follower(102, 200)
    assert r.rl_follower_count() == 3
    for nid, v, tick in [(100, 1, 0), (101, 4, 2), (102, 200, 2)]:
        assert r.rl_follower_size(nid) == v
        assert r.rl_follower_tick(nid) == tick


def test_gc_remove_out_of_date_follower_state():  # rate_test.go:102-128
    r = _rl(100)
    r.rl_set_follower(101, 1)
    r.rl_heartbeat_tick()
    r.rl_set_follower(102, 2)
    r.rl_set_follower(103, 3)
    r.rl_gc()
    assert r.rl_follower_count() == 3
    r.rl_heartbeat_tick()
    r.rl_heartbeat_tick()
    r.rl_gc()
    assert r.rl_follower_count() == 2
    assert r.rl_follower_size(101) == -1
    r.rl_heartbeat_tick()
    r.rl_gc()
    assert r.rl_follower_count() == 0


def test_rate_limited():  # rate_test.go:130-140
    r = _rl(100)
    r.rl_increase(100)
    assert not r.rl_rate_limited()
    r.rl_increase(1)
    assert r.rl_rate_limited()


def test_rate_limited_when_follower_is_rate_limited():  # rate_test.go:142-153
    r = _rl(100)
    r.rl_increase(100)
    assert not r.rl_rate_limited()
    r.rl_set_follower(1, 100)
    r.rl_set_follower(2, 101)
    assert r.rl_rate_limited()


def test_rate_not_limited_when_out_of_date_follower_state_is_limited():  # rate_test.go:155-173
    r = _rl(100)
    r.rl_increase(100)
    assert not r.rl_rate_limited()
    r.rl_set_follower(1, 100)
    r.rl_set_follower(2, 101)
    for _ in range(4):
        r.rl_heartbeat_tick()
    assert not r.rl_rate_limited()
    assert r.rl_follower_count() == 0  # GCed by RateLimited


def test_not_enabled_rate_limit_never_limit_rates():  # rate_test.go:175-183
    r = _rl(0)
    for _ in range(10000):
        r.rl_increase(U64_MAX // 2)
        assert not r.rl_rate_limited()


def test_reset_follower_state():  # rate_test.go:185-196
    r = _rl(1024)
    r.rl_set_follower(1, 1025)
    assert r.rl_rate_limited()
    r.rl_reset_followers()
    assert not r.rl_rate_limited()


# ------------------------------------------------------- inmemory_test.go
def _im_rl(marker_last, max_size):
    """newInMemory(lastIndex, server.NewRateLimiter(max_size))."""
    im = InMem(marker_last + 1, [], saved_to=marker_last)
    im.op(11, max_size)
    return im


def _merge_cmds(im, ents):
    a = [O.Entry(index=i, term=0, cmd=bytes(n)) for i, n in ents]
    arr = O.entries_array(a)
    assert im.L.orc_inmem_merge(im.h, arr, len(a)) == 0


@pytest.mark.parametrize("max_size,limited", [(None, False), (0, False), (U64_MAX, False),
                                              (1, True), (U64_MAX - 1, True)])
def test_inmem_rate_limited(max_size, limited):  # inmemory_test.go:558-575
    im = InMem(1, [])
    if max_size is not None:
        im.op(11, max_size)
    # rateLimited() == rl != nil && rl.Enabled(): observed through merge's Increase
    _merge_cmds(im, [(1, 8)])
    got = im.op(12)
    assert (got == in_mem_size([8])) == limited
    if max_size is not None and not limited:
        assert got == 0


def test_rate_limit_cleared_after_restoring_snapshot():  # inmemory_test.go:577-587
    im = _im_rl(0, 10000)
    _merge_cmds(im, [(0, 1024)])
    assert im.op(12) != 0
    im.op(9, 0, 0)
    assert im.op(12) == 0


def test_rate_limit_is_updated_after_merging_entries():  # inmemory_test.go:589-602
    im = _im_rl(0, 10000)
    _merge_cmds(im, [(1, 1024)])
    logsz = im.op(12)
    _merge_cmds(im, [(2, 16), (3, 64)])
    assert im.op(12) == logsz + in_mem_size([16, 64])


def test_rate_limit_is_decreased_after_entries_are_applied():  # inmemory_test.go:604-626
    sizes = {2: 16, 3: 64, 4: 128}
    im = _im_rl(2, 10000)
    _merge_cmds(im, list(sizes.items()))
    assert im.op(12) == in_mem_size(sizes.values())
    for idx in range(2, 5):
        im.op(1, idx)
        # entries[1:] are the ones still counted
        assert im.first == idx
        assert im.op(12) == in_mem_size([sizes[i] for i in range(idx + 1, 5)])


def test_rate_limit_can_be_reset_when_merging_entries():  # inmemory_test.go:628-644
    im = _im_rl(2, 10000)
    _merge_cmds(im, [(2, 16), (3, 64), (4, 128)])
    _merge_cmds(im, [(1, 16)])
    assert im.op(12) == in_mem_size([16])


def test_rate_limit_can_be_updated_after_cut_and_merging_entries():  # inmemory_test.go:646-660
    im = _im_rl(2, 10000)
    _merge_cmds(im, [(2, 16), (3, 64), (4, 128)])
    _merge_cmds(im, [(3, 1024), (4, 1024)])
    assert im.op(12) == in_mem_size([16, 1024, 1024])


# ----------------------------------------------------------- raft_test.go
def _rate_limited_raft():
    """newRateLimitedTestRaft(1, {1,2,3}, 5, 1) (raft_etcd_test.go:3005-3020)."""
    r = O.Raft.new(1, [1, 2, 3], election=5, heartbeat=1)
    r.rl_set_max(TEST_RATE_LIMIT)
    return r


@pytest.mark.parametrize("is_leader", [True, False])
def test_node_updates_its_rate_limiter_heartbeat(is_leader):  # raft_test.go:2783-2807
    r = _rate_limited_raft()
    if is_leader:
        r.become_candidate()
        r.become_leader()
    else:
        r.become_follower(0, 2)
    hbt = r.rl_tick()
    for _ in range(r.election_timeout):
        r.tick()
    assert r.rl_tick() == hbt + 1


def test_reset_clears_follower_rate_limit_state():  # raft_test.go:2809-2820
    r = _rate_limited_raft()
    r.rl_handle_leader_rate_limit(2, TEST_RATE_LIMIT + 1)
    assert r.rl_rate_limited()
    r.reset(2)
    assert not r.rl_rate_limited()


def test_leader_rate_limit_message_is_handled_by_leader():  # raft_test.go:2822-2832
    r = _rate_limited_raft()
    assert not r.rl_rate_limited()
    r.rl_handle_leader_rate_limit(2, TEST_RATE_LIMIT + 1)
    assert r.rl_rate_limited()


def _rate_limit_msgs(r):
    return [m for m in r.read_messages() if m.type == O.RateLimit]


def test_rate_limit_message_is_never_sent_by_leader():  # raft_test.go:2834-2855
    r = _rate_limited_raft()
    r.become_candidate()
    r.become_leader()
    r.rl_append_entries(0, TEST_RATE_LIMIT + 1)
    assert r.rl_rate_limited()
    for _ in range(r.election_timeout):
        r.tick()
    assert not _rate_limit_msgs(r)


@pytest.mark.parametrize("leader,sent", [(2, True), (0, False)])
def test_rate_limit_message_is_sent_by_non_leader(leader, sent):  # raft_test.go:2857-2885
    r = _rate_limited_raft()
    r.become_follower(2, leader)
    r.rl_append_entries(0, TEST_RATE_LIMIT + 1)
    assert r.rl_rate_limited()
    for _ in range(r.election_timeout):
        r.tick()
    msgs = _rate_limit_msgs(r)
    assert bool(msgs) == sent
    if sent:
        m = msgs[0]
        assert m.to == 2 and m.term == 2
        # Hint: inmem size less the uncommitted entries' SizeUpperLimit (wraps
        # as uint64 when the latter is larger, raft.go:672-676)
        inmem = in_mem_size([TEST_RATE_LIMIT + 1])
        upper = 128 + TEST_RATE_LIMIT + 1
        assert m.hint == (inmem - upper) % (1 << 64)


def test_rate_limit_disabled_sends_nothing():  # raft.go:571-576 with rl.Enabled() false
    r = O.Raft.new(1, [1, 2, 3], election=5, heartbeat=1)
    r.become_follower(2, 2)
    for _ in range(3 * r.election_timeout):
        r.tick()
    assert not _rate_limit_msgs(r)
    assert r.rl_tick() == 0
