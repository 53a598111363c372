// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of dragonboat's internal/raft (github.com/lni/dragonboat/v3,
// mounted at /root/reference) used as the parity checker for the MI355X batched
// Raft step engine.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it; the product path (dragonboat_amd/) never does.
//
// Pinning: the restatement is checked against the reference's own table-driven
// tests (internal/raft/*_test.go), transcribed into tests/test_oracle_*.py.
// The Go toolchain is absent from this image, so the reference itself cannot be
// built or run here; those transcribed known-answer tests are the
// pin.
//
// Semantics follow the Go code function by function; every function cites the
// reference file:line it restates.  Go maps are replaced by std::map, whose
// ascending-key iteration is the canonical order used everywhere (the Go code
// iterates maps in random order; state transitions are order-independent and the
// message stream is defined per destination).
// The randomized election timeout source (goutils random.LockGuardedRand,
// raft.go:632) is replaced by an injected counter-based PRNG (rto_rand below).
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

namespace orc {

using u64 = uint64_t;
using u32 = uint32_t;

// raftpb/raft.pb.go:23-51
enum MessageType : int {
  LocalTick = 0, Election = 1, LeaderHeartbeat = 2, ConfigChangeEvent = 3,
  NoOP = 4, Ping = 5, Pong = 6, Propose = 7, SnapshotStatus = 8,
  Unreachable = 9, CheckQuorum = 10, BatchedReadIndex = 11, Replicate = 12,
  ReplicateResp = 13, RequestVote = 14, RequestVoteResp = 15,
  InstallSnapshot = 16, Heartbeat = 17, HeartbeatResp = 18, ReadIndex = 19,
  ReadIndexResp = 20, Quiesce = 21, SnapshotReceived = 22,
  LeaderTransfer = 23, TimeoutNow = 24, RateLimit = 25,
  NumMessageTypes = 26  // raft.go:49
};

// raftpb/raft.pb.go:138-141
enum EntryType : int { ApplicationEntry = 0, ConfigChangeEntry = 1,
                       EncodedEntry = 2, MetadataEntry = 3 };
// raftpb/raft.pb.go:184-187
enum ConfigChangeType : int { AddNode = 0, RemoveNode = 1, AddObserver = 2,
                              AddWitness = 3 };

// raft.go:63-70
enum State : int { Follower = 0, Candidate = 1, Leader = 2, Observer = 3,
                   Witness = 4, NumStates = 5 };

// remote.go:27-32
enum RemoteState : int { RemoteRetry = 0, RemoteWait = 1, RemoteReplicate = 2,
                         RemoteSnapshot = 3 };

constexpr u64 NoLeader = 0;
constexpr u64 NoNode = 0;
constexpr u64 NoLimit = ~0ULL;
constexpr u64 EntryNonCmdFieldsSize = 16 * 8;  // internal/settings/soft.go:20
constexpr u64 DefaultMaxEntrySize = 64ULL * 1024 * 1024;  // soft.go:226 (LargeEntitySize)
constexpr u64 InMemGCTimeout = 100;  // soft.go:227

struct Panic : std::runtime_error {
  explicit Panic(const std::string& s) : std::runtime_error(s) {}
};
[[noreturn]] void panicf(const char* fmt, ...);

// splitmix64: the counter-based mixer shared by the oracle and the device
// engine for every injected random value (election timeouts, workloads).
inline u64 splitmix64(u64 x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
// Uniform draw in [0, m) from the high 32 bits of x (multiply-shift).  The
// reference computes Uint64() % electionTimeout; the injected source is ours
// to define, and this form needs no 64-bit division on device.
inline u64 below(u64 x, u64 m) { return ((x >> 32) * (m & 0xFFFFFFFFULL)) >> 32; }
// Injected replacement for random.LockGuardedRand.Uint64() at raft.go:632.
inline u64 rto_rand(u64 seed, u64 cid, u64 nid, u64 count) {
  return splitmix64(seed ^ (cid * 0x9E3779B97F4A7C15ULL) ^ (nid << 32) ^ count);
}

// raftpb Entry (raft.pb.go:589-598)
struct Entry {
  u64 term = 0;
  u64 index = 0;
  int type = ApplicationEntry;
  u64 key = 0, client_id = 0, series_id = 0, responded_to = 0;
  std::string cmd;
  // raftpb/raft_optimized.go:72-76
  u64 sizeUpperLimit() const { return EntryNonCmdFieldsSize + cmd.size(); }
};

struct SystemCtx {  // raftpb/raft.go:45-49
  u64 low = 0, high = 0;
  bool operator==(const SystemCtx& o) const { return low == o.low && high == o.high; }
  bool operator!=(const SystemCtx& o) const { return !(*this == o); }
  bool operator<(const SystemCtx& o) const {
    return low < o.low || (low == o.low && high < o.high);
  }
};

struct Membership {  // raft.pb.go:733-739
  u64 config_change_id = 0;
  std::map<u64, std::string> addresses;
  std::map<u64, bool> removed;
  std::map<u64, std::string> observers;
  std::map<u64, std::string> witnesses;
};

struct Snapshot {  // raft.pb.go:879-893 (the fields the raft core reads)
  std::string filepath;
  u64 file_size = 0;
  u64 index = 0;
  u64 term = 0;
  Membership membership;
  bool dummy = false;
  u64 cluster_id = 0;
  bool witness = false;
  int files = 0;
};
inline bool isEmptySnapshot(const Snapshot& s) { return s.index == 0; }  // raftpb/raft.go:132

struct Message {  // raft.pb.go:1019-1033
  int type = LocalTick;
  u64 to = 0, from = 0, cluster_id = 0, term = 0, log_term = 0, log_index = 0,
      commit = 0;
  bool reject = false;
  u64 hint = 0;
  std::vector<Entry> entries;
  Snapshot snapshot;
  u64 hint_high = 0;
};

struct PState {  // raftpb State, raft.pb.go:529-533
  u64 term = 0, vote = 0, commit = 0;
};
inline bool isStateEqual(const PState& a, const PState& b) {  // raftpb/raft.go:141
  return a.term == b.term && a.vote == b.vote && a.commit == b.commit;
}
inline bool isEmptyState(const PState& s) { return isStateEqual(s, PState{}); }

struct ReadyToRead {  // raftpb/raft.go:52-56
  u64 index = 0;
  SystemCtx ctx;
};

struct UpdateCommit {  // raftpb/raft.go:60-70
  u64 processed = 0, last_applied = 0, stable_log_to = 0, stable_log_term = 0,
      stable_snapshot_to = 0, ready_to_read = 0;
};

struct Update {  // raftpb/raft.go:74-110
  u64 cluster_id = 0, node_id = 0;
  PState state;
  bool fast_apply = false;
  std::vector<Entry> entries_to_save;
  std::vector<Entry> committed_entries;
  bool more_committed_entries = false;
  Snapshot snapshot;
  std::vector<ReadyToRead> ready_to_reads;
  std::vector<Message> messages;
  u64 last_applied = 0;
  UpdateCommit update_commit;
  std::vector<Entry> dropped_entries;
  std::vector<SystemCtx> dropped_read_indexes;
};

enum Err : int { ErrOK = 0, ErrCompacted = 1, ErrUnavailable = 2,
                 ErrSnapshotOutOfDate = 3 };

// entryutils.go:73-111
bool isLocalMessageType(int t);
bool isResponseMessageType(int t);
int countConfigChange(const std::vector<Entry>& ents);  // entryutils.go:23-31
void checkEntriesToAppend(const std::vector<Entry>& ents,
                          const std::vector<Entry>& toAppend);  // entryutils.go:38-50
std::vector<Entry> limitSize(const std::vector<Entry>& ents, u64 limit);  // entryutils.go:52-64

// ILogDB, logentry.go:45-73
struct ILogDB {
  virtual ~ILogDB() {}
  virtual std::pair<u64, u64> GetRange() = 0;
  virtual void SetRange(u64 index, u64 length) = 0;
  virtual std::pair<PState, Membership> NodeState() = 0;
  virtual void SetState(const PState& ps) = 0;
  virtual Err CreateSnapshot(const Snapshot& ss) = 0;
  virtual Err ApplySnapshot(const Snapshot& ss) = 0;
  virtual Err Term(u64 index, u64* term) = 0;
  virtual Err Entries(u64 low, u64 high, u64 maxSize, std::vector<Entry>* out) = 0;
  virtual Snapshot GetSnapshot() = 0;
  virtual Err Compact(u64 index) = 0;
  virtual Err Append(const std::vector<Entry>& entries) = 0;
};

// TestLogDB, internal/raft/logdb_test.go:25-177: the in-memory ILogDB the
// reference's raft tests use; also the LogDB of the lockstep harness.
struct TestLogDB : ILogDB {
  std::vector<Entry> entries;
  u64 markerIndex = 0;
  u64 markerTerm = 0;
  Snapshot snapshot;
  PState state;

  std::pair<u64, u64> GetRange() override { return {firstIndex(), lastIndex()}; }
  u64 firstIndex() const { return markerIndex + 1; }
  u64 lastIndex() const { return markerIndex + entries.size(); }
  void SetRange(u64, u64) override { panicf("not implemented"); }
  std::pair<PState, Membership> NodeState() override { return {state, snapshot.membership}; }
  void SetState(const PState& s) override { state = s; }
  Err CreateSnapshot(const Snapshot& ss) override;
  Err ApplySnapshot(const Snapshot& ss) override;
  Err Term(u64 index, u64* term) override;
  Err Entries(u64 low, u64 high, u64 maxSize, std::vector<Entry>* out) override;
  Snapshot GetSnapshot() override { return snapshot; }
  Err Compact(u64 index) override;
  Err Append(const std::vector<Entry>& entries) override;
};

// internal/server/rate.go:33-137: the in-memory log size limiter.  Go's
// follower map holds (tick, inMemLogSize) per follower; gc() drops the states
// older than gcTick heartbeat ticks.
constexpr u64 RateLimitGcTick = 2;  // rate.go:25 gcTick
struct RateLimiter {
  u64 size = 0;
  u64 tick = 0;
  u64 maxSize = 0;
  std::map<u64, std::pair<u64, u64>> followerSizes;  // nodeID -> (tick, inMemLogSize)

  bool enabled() const { return maxSize > 0 && maxSize != ~0ull; }  // rate.go:59-61
  void heartbeatTick() { tick++; }                                    // rate.go:64-66
  void increase(u64 sz) { size += sz; }                               // rate.go:74-76
  void decrease(u64 sz) { size -= sz; }  // rate.go:79-81 (AddUint64 of ^(sz-1): wraps)
  void set(u64 sz) { size = sz; }
  u64 get() const { return size; }
  void resetFollowerState() { followerSizes.clear(); }              // rate.go:94-96
  void setFollowerState(u64 nodeID, u64 sz) { followerSizes[nodeID] = {tick, sz}; }
  bool rateLimited();                                                 // rate.go:109-111
  void gc();                                                          // rate.go:139-149
};
// raftpb/raft.go:301-322: SizeUpperLimit sum, and the in-memory size (Cmd
// bytes + unsafe.Sizeof(pb.Entry) = 80 on 64-bit Go: 7 words + a slice header)
constexpr u64 GoEntryStructSize = 80;
u64 entrySliceSize(const std::vector<Entry>& ents);
u64 entrySliceInMemSize(const std::vector<Entry>& ents);

// inmemory.go:36-44
struct InMemory {
  bool shrunk = false;
  bool newEntries = true;
  bool hasSnapshot = false;
  Snapshot snapshot;
  std::vector<Entry> entries;
  u64 markerIndex = 0;
  u64 savedTo = 0;
  RateLimiter* rl = nullptr;  // the raft's limiter (newEntryLog(logdb, rl))

  bool rateLimited() const { return rl != nullptr && rl->enabled(); }  // inmemory.go:248-250
  void init(u64 lastIndex);  // newInMemory, inmemory.go:46-57
  void checkMarkerIndex() const;
  std::vector<Entry> getEntries(u64 low, u64 high) const;
  bool getSnapshotIndex(u64* idx) const;
  bool getLastIndex(u64* idx) const;
  bool getTerm(u64 index, u64* term) const;
  void commitUpdate(const UpdateCommit& cu);
  std::vector<Entry> entriesToSave() const;
  void savedLogTo(u64 index, u64 term);
  void appliedLogTo(u64 index);
  void savedSnapshotTo(u64 index);
  void resize() { shrunk = false; }
  void tryResize() { if (shrunk) resize(); }
  void resizeEntrySlice();
  void merge(const std::vector<Entry>& ents);
  void restore(const Snapshot& ss);
};

// logentry.go:78-84
struct EntryLog {
  ILogDB* logdb = nullptr;
  InMemory inmem;
  u64 committed = 0;
  u64 processed = 0;
  u64 maxEntrySize = DefaultMaxEntrySize;  // settings.Soft.MaxEntrySize

  void init(ILogDB* db);  // newEntryLog, logentry.go:86-96
  u64 firstIndex() const;
  u64 lastIndex() const;
  std::pair<u64, u64> termEntryRange() const;
  bool entryRange(u64* first, u64* last) const;
  u64 lastTerm() const;
  Err term(u64 index, u64* t) const;
  Err checkBound(u64 low, u64 high) const;
  std::vector<Entry> getUncommittedEntries() const;
  Err getEntriesFromLogDB(u64 low, u64 high, u64 maxSize, std::vector<Entry>* ents,
                          bool* checkInMem) const;
  std::vector<Entry> getEntriesFromInMem(std::vector<Entry> ents, u64 low, u64 high) const;
  Err getEntries(u64 low, u64 high, u64 maxSize, std::vector<Entry>* out) const;
  Err entries(u64 start, u64 maxSize, std::vector<Entry>* out) const;
  Snapshot snapshot() const;
  u64 firstNotAppliedIndex() const;
  u64 toApplyIndexLimit() const { return committed + 1; }
  bool hasEntriesToApply() const;
  bool hasMoreEntriesToApply(u64 appliedTo) const { return committed > appliedTo; }
  std::vector<Entry> entriesToApply() const { return getEntriesToApply(maxEntrySize); }
  std::vector<Entry> getEntriesToApply(u64 limit) const;
  std::vector<Entry> entriesToSave() const { return inmem.entriesToSave(); }
  bool tryAppend(u64 index, const std::vector<Entry>& ents);
  void append(const std::vector<Entry>& entries);
  u64 getConflictIndex(const std::vector<Entry>& entries) const;
  void commitTo(u64 index);
  void commitUpdate(const UpdateCommit& cu);
  bool matchTerm(u64 index, u64 term) const;
  bool upToDate(u64 index, u64 term) const;
  bool tryCommit(u64 index, u64 term);
  void restore(const Snapshot& s);
};

// remote.go:62-69
struct Remote {
  u64 match = 0;
  u64 next = 0;
  u64 snapshotIndex = 0;
  int state = RemoteRetry;
  bool active = false;

  void reset() { snapshotIndex = 0; }
  void becomeRetry();
  void retryToWait() { if (state == RemoteRetry) state = RemoteWait; }
  void waitToRetry() { if (state == RemoteWait) state = RemoteRetry; }
  void becomeWait() { becomeRetry(); retryToWait(); }
  void becomeReplicate();
  void becomeSnapshot(u64 index);
  void clearPendingSnapshot() { snapshotIndex = 0; }
  bool tryUpdate(u64 index);
  void progress(u64 lastIndex);
  void respondedTo();
  bool decreaseTo(u64 rejected, u64 last);
  bool isPaused() const;
  bool isActive() const { return active; }
  void setActive() { active = true; }
  void setNotActive() { active = false; }
};

// readindex.go:24-34
struct ReadStatus {
  u64 index = 0;
  u64 from = 0;
  SystemCtx ctx;
  std::set<u64> confirmed;
};
struct ReadIndexQ {
  std::map<SystemCtx, ReadStatus> pending;
  std::vector<SystemCtx> queue;
  void addRequest(u64 index, SystemCtx ctx, u64 from);
  bool hasPendingRequest() const { return !queue.empty(); }
  SystemCtx peepCtx() const { return queue.back(); }
  std::vector<ReadStatus> confirm(SystemCtx ctx, u64 from, int quorum);
};

// config.Config (config/config.go:60-171), the fields the raft core reads
struct Config {
  u64 nodeID = 0;
  u64 clusterID = 0;
  u64 electionRTT = 0;
  u64 heartbeatRTT = 0;
  bool checkQuorum = false;
  bool quiesce = false;
  bool isObserver = false;
  bool isWitness = false;
  u64 maxInMemLogSize = 0;  // rate limiter (server.NewRateLimiter), 0 = disabled
  u64 rngSeed = 0x5EEDD8A6ULL;  // injected PRNG seed (replaces goutils random)
  u64 maxEntrySize = DefaultMaxEntrySize;
};

// events recorded from server.IRaftEventListener (internal/server/event.go)
struct Events {
  u64 leaderUpdated = 0, campaignLaunched = 0, campaignSkipped = 0,
      snapshotRejected = 0, replicationRejected = 0, proposalDropped = 0,
      readIndexDropped = 0;
};

// raft.go:197-232
struct Raft {
  u64 applied = 0;
  u64 nodeID = 0;
  u64 clusterID = 0;
  u64 term = 0;
  u64 vote = 0;
  EntryLog log;
  std::map<u64, Remote> remotes;
  std::map<u64, Remote> observers;
  std::map<u64, Remote> witnesses;
  int state = Follower;
  std::map<u64, bool> votes;
  std::vector<Message> msgs;
  u64 leaderID = NoLeader;
  u64 leaderTransferTarget = NoNode;
  bool isLeaderTransferTarget = false;
  bool pendingConfigChange = false;
  ReadIndexQ readIndex;
  std::vector<ReadyToRead> readyToRead;
  std::vector<Entry> droppedEntries;
  std::vector<SystemCtx> droppedReadIndexes;
  bool quiesce = false;
  bool checkQuorum = false;
  u64 tickCount = 0;
  u64 electionTick = 0;
  u64 heartbeatTick = 0;
  u64 heartbeatTimeout = 0;
  u64 electionTimeout = 0;
  u64 randomizedElectionTimeout = 0;
  std::vector<u64> matched;
  bool testOnlyCCMode = false;  // hasNotAppliedConfigChange test hook
  Events events;
  bool hasEvents = true;
  u64 rngSeed = 0;
  u64 rngCount = 0;  // number of randomized timeouts drawn so far
  u64 maxEntrySize = DefaultMaxEntrySize;
  RateLimiter rl;  // raft.go:204; the in-memory log reports its size to it

  Raft(const Config& c, ILogDB* logdb);  // newRaft, raft.go:234-289
  void setTestPeers(const std::vector<u64>& peers);
  u64 numVotingMembers() const { return remotes.size() + witnesses.size(); }
  int quorum() const { return (int)numVotingMembers() / 2 + 1; }
  bool isSingleNodeQuorum() const { return quorum() == 1; }
  bool isLeader() const { return state == Leader; }
  bool isCandidate() const { return state == Candidate; }
  bool isObserver() const { return state == Observer; }
  bool isWitness() const { return state == Witness; }
  void mustBeLeader() const;
  void setLeaderID(u64 leaderID);
  bool leaderTransfering() const { return leaderTransferTarget != NoNode && isLeader(); }
  void abortLeaderTransfer() { leaderTransferTarget = NoNode; }
  bool leaderHasQuorum();
  std::vector<u64> nodes() const;
  std::vector<u64> nodesSorted() const;
  std::map<u64, Remote*> votingMembers();
  PState raftState() const { return PState{term, vote, log.committed}; }
  void loadState(const PState& st);
  bool restore(const Snapshot& ss);
  void restoreRemotes(const Snapshot& ss);
  bool timeForElection() const { return electionTick >= randomizedElectionTimeout; }
  bool timeForHearbeat() const { return heartbeatTick >= heartbeatTimeout; }
  bool timeForCheckQuorum() const { return electionTick >= electionTimeout; }
  bool timeToAbortLeaderTransfer() const { return leaderTransfering() && electionTick >= electionTimeout; }
  bool timeForRateLimitCheck() const { return tickCount % electionTimeout == 0; }
  bool timeForInMemGC() const { return tickCount % InMemGCTimeout == 0; }
  void tick();
  void nonLeaderTick();
  void leaderTick();
  void quiescedTick();
  void setRandomizedElectionTimeout();
  Message finalizeMessageTerm(Message m) const;
  void send(Message m);
  void makeInstallSnapshotMessage(u64 to, Message* m, u64* index);
  Err makeReplicateMessage(u64 to, u64 next, u64 maxSize, Message* out);
  void sendReplicateMessage(u64 to);
  void broadcastReplicateMessage();
  void sendHeartbeatMessage(u64 to, SystemCtx hint, u64 match);
  void broadcastHeartbeatMessage();
  void broadcastHeartbeatMessageWithHint(SystemCtx ctx);
  void sendTimeoutNowMessage(u64 nodeID);
  void sendRateLimitMessage();  // raft.go:660-683
  void sortMatchValues();
  bool tryCommit();
  void appendEntries(std::vector<Entry> entries);
  void becomeObserver(u64 term, u64 leaderID);
  void becomeWitness(u64 term, u64 leaderID);
  void becomeFollower(u64 term, u64 leaderID);
  void becomeCandidate();
  void becomeLeader();
  void reset(u64 term);
  void preLeaderPromotionHandleConfigChange();
  void resetRemotes();
  void resetObservers();
  void resetWitnesses();
  void resetMatchValueArray() { matched.assign(numVotingMembers(), 0); }
  int handleVoteResp(u64 from, bool rejected);
  void campaign();
  bool selfRemoved() const;
  void addNode(u64 nodeID);
  void addObserver(u64 nodeID);
  void addWitness(u64 nodeID);
  void removeNode(u64 nodeID);
  void setRemote(u64 nodeID, u64 match, u64 next);
  void setObserver(u64 nodeID, u64 match, u64 next);
  void setWitness(u64 nodeID, u64 match, u64 next);
  int getPendingConfigChangeCount();
  bool hasConfigChangeToApply();
  bool testOnlyHasConfigChangeToApply();
  bool canGrantVote(const Message& m) const {
    return vote == NoNode || vote == m.from || m.term > term;
  }
  bool dropRequestVoteFromHighTermNode(const Message& m);
  bool onMessageTermNotMatched(const Message& m);
  void doubleCheckTermMatched(u64 msgTerm) const;
  bool hasCommittedEntryAtCurrentTerm() const;
  void addReadyToRead(u64 index, SystemCtx ctx) { readyToRead.push_back({index, ctx}); }
  void enterRetryState(Remote* rp) { if (rp->state == RemoteReplicate) rp->becomeRetry(); }
  void reportDroppedConfigChange(const Entry& e) { droppedEntries.push_back(e); }
  void reportDroppedProposal(const Message& m);
  void reportDroppedReadIndex(const Message& m);
  Remote* lookupRemote(u64 from);  // lw(), raft.go:2014-2028

  // message handlers (raft.go:1301-1981)
  void Handle(Message m);  // raft.go:1451-1458
  void dispatch(Message& m);  // defaultHandle + initializeHandlerMap, raft.go:2030-2098
  void handleHeartbeatMessage(const Message& m);
  void handleInstallSnapshotMessage(const Message& m);
  void handleReplicateMessage(const Message& m);
  void handleNodeElection(const Message& m);
  void handleNodeRequestVote(const Message& m);
  void handleNodeConfigChange(const Message& m);
  void handleLocalTick(const Message& m);
  void handleRestoreRemote(const Message& m);
  void handleLeaderHeartbeat(const Message& m);
  void handleLeaderCheckQuorum(const Message& m);
  void handleLeaderPropose(Message& m);
  void handleLeaderReadIndex(const Message& m);
  void handleLeaderReplicateResp(const Message& m, Remote* rp);
  void handleLeaderHeartbeatResp(const Message& m, Remote* rp);
  void handleLeaderTransfer(const Message& m, Remote* rp);
  void handleReadIndexLeaderConfirmation(const Message& m);
  void handleLeaderSnapshotStatus(const Message& m, Remote* rp);
  void handleLeaderUnreachable(const Message& m, Remote* rp);
  void handleLeaderRateLimit(const Message& m);
  void handleFollowerPropose(Message& m);
  void handleFollowerReplicate(const Message& m);
  void handleFollowerHeartbeat(const Message& m);
  void handleFollowerReadIndex(Message& m);
  void handleFollowerLeaderTransfer(Message& m);
  void handleFollowerReadIndexResp(const Message& m);
  void handleFollowerInstallSnapshot(const Message& m);
  void handleFollowerTimeoutNow(const Message& m);
  void handleCandidatePropose(const Message& m);
  void handleCandidateReadIndex(const Message& m);
  void handleCandidateReplicate(const Message& m);
  void handleCandidateInstallSnapshot(const Message& m);
  void handleCandidateHeartbeat(const Message& m);
  void handleCandidateRequestVoteResp(const Message& m);

  std::vector<Message> readMessages() {  // raft_etcd_test.go:119-124
    std::vector<Message> out;
    out.swap(msgs);
    return out;
  }
};

// Peer API, peer.go:58-358
struct Peer {
  Raft* raft = nullptr;
  PState prevState;
  bool rateLimited() { return raft->rl.rateLimited(); }  // peer.go:245-249

  ~Peer() { delete raft; }
  static Peer* Launch(const Config& c, ILogDB* logdb,
                      const std::vector<std::pair<u64, std::string>>& addresses,
                      bool initial, bool newNode);
  void Tick();
  void QuiescedTick();
  void RequestLeaderTransfer(u64 target);
  void ProposeEntries(const std::vector<Entry>& ents);
  void ProposeConfigChange(const std::string& data, u64 key);  // data: the marshaled ConfigChange
  void ApplyConfigChange(u64 nodeID, int ccType);
  void RejectConfigChange();
  void RestoreRemotes(const Snapshot& ss);
  void ReportUnreachableNode(u64 nodeID);
  void ReportSnapshotStatus(u64 nodeID, bool reject);
  void Handle(const Message& m);
  Update GetUpdate(bool moreToApply, u64 lastApplied);
  bool HasUpdate(bool moreEntriesToApply) const;
  void Commit(const Update& ud);
  void ReadIndex(SystemCtx ctx);
  void NotifyRaftLastApplied(u64 lastApplied) { raft->applied = lastApplied; }
  bool HasEntryToApply() const { return raft->log.hasEntriesToApply(); }
  Update getUpdate(bool moreEntriesToApply, u64 lastApplied) const;
};
Update setFastApply(Update ud);  // peer.go:209-226
void validateUpdate(const Update& ud);  // peer.go:228-245
UpdateCommit getUpdateCommit(const Update& ud);  // peer.go:410-427
void bootstrap(Raft* r, std::vector<std::pair<u64, std::string>> addresses);  // peer.go:378-408

}  // namespace orc
