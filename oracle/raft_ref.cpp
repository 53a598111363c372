// ORACLE — TEST INFRASTRUCTURE ONLY (see raft_ref.h header comment).
// CPU restatement of /root/reference/internal/raft/{raft,remote,readindex,
// logentry,inmemory,entryutils,peer}.go and logdb_test.go's TestLogDB.
#include "raft_ref.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>

namespace orc {

void panicf(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw Panic(buf);
}

static inline u64 umin(u64 a, u64 b) { return a > b ? b : a; }  // entryutils.go:66-71
static inline u64 umax(u64 a, u64 b) { return a > b ? a : b; }  // entryutils.go:73-78

// ---------------------------------------------------------------- entryutils.go
int countConfigChange(const std::vector<Entry>& ents) {  // entryutils.go:23-31
  int c = 0;
  for (auto& e : ents)
    if (e.type == ConfigChangeEntry) c++;
  return c;
}

void checkEntriesToAppend(const std::vector<Entry>& ents,
                          const std::vector<Entry>& toAppend) {  // entryutils.go:38-50
  if (ents.empty() || toAppend.empty()) return;
  if (ents.back().index + 1 != toAppend[0].index)
    panicf("found a hole, last %llu, first to append %llu",
           (unsigned long long)ents.back().index, (unsigned long long)toAppend[0].index);
  if (ents.back().term > toAppend[0].term)
    panicf("term value not expected, %llu vs %llu", (unsigned long long)ents.back().term,
           (unsigned long long)toAppend[0].term);
}

std::vector<Entry> limitSize(const std::vector<Entry>& ents, u64 limit) {  // entryutils.go:52-64
  if (ents.empty()) return ents;
  u64 total = ents[0].sizeUpperLimit();
  size_t inc;
  for (inc = 1; inc < ents.size(); inc++) {
    total += ents[inc].sizeUpperLimit();
    if (total > limit) break;
  }
  return std::vector<Entry>(ents.begin(), ents.begin() + inc);
}

bool isLocalMessageType(int t) {  // entryutils.go:89-97
  return t == Election || t == LeaderHeartbeat || t == Unreachable ||
         t == SnapshotStatus || t == CheckQuorum || t == LocalTick ||
         t == BatchedReadIndex;
}

bool isResponseMessageType(int t) {  // entryutils.go:99-107
  return t == ReplicateResp || t == RequestVoteResp || t == HeartbeatResp ||
         t == ReadIndexResp || t == Unreachable || t == SnapshotStatus ||
         t == LeaderTransfer;
}

// ---------------------------------------------------------------- TestLogDB
Err TestLogDB::ApplySnapshot(const Snapshot& ss) {  // logdb_test.go:51-60
  if (snapshot.index >= ss.index) return ErrSnapshotOutOfDate;
  snapshot = ss;
  markerIndex = ss.index;
  markerTerm = ss.term;
  entries.clear();
  return ErrOK;
}

Err TestLogDB::CreateSnapshot(const Snapshot& ss) {  // logdb_test.go:62-68
  if (snapshot.index >= ss.index) return ErrSnapshotOutOfDate;
  snapshot = ss;
  return ErrOK;
}

Err TestLogDB::Term(u64 index, u64* term) {  // logdb_test.go:107-119
  if (index == markerIndex) {
    *term = markerTerm;
    return ErrOK;
  }
  std::vector<Entry> ents;
  Err err = Entries(index, index + 1, NoLimit, &ents);
  if (err != ErrOK) {
    *term = 0;
    return err;
  }
  *term = ents.empty() ? 0 : ents[0].term;
  return ErrOK;
}

Err TestLogDB::Append(const std::vector<Entry>& in) {  // logdb_test.go:121-141
  if (in.empty()) return ErrOK;
  std::vector<Entry> ents = in;
  u64 first = firstIndex();
  if (markerIndex + ents.size() < first) return ErrOK;
  if (first > ents[0].index) ents.erase(ents.begin(), ents.begin() + (first - ents[0].index));
  u64 offset = ents[0].index - markerIndex;
  if ((u64)entries.size() + 1 > offset) {
    entries.resize(offset - 1);
  } else if ((u64)entries.size() + 1 < offset) {
    panicf("found a hole last index %llu, first incoming index %llu",
           (unsigned long long)lastIndex(), (unsigned long long)ents[0].index);
  }
  entries.insert(entries.end(), ents.begin(), ents.end());
  return ErrOK;
}

Err TestLogDB::Entries(u64 low, u64 high, u64 maxSize,
                       std::vector<Entry>* out) {  // logdb_test.go:143-157
  out->clear();
  if (low <= markerIndex) return ErrCompacted;
  if (high > lastIndex() + 1) return ErrUnavailable;
  if (entries.empty()) return ErrUnavailable;
  std::vector<Entry> ents(entries.begin() + (low - markerIndex - 1),
                          entries.begin() + (high - markerIndex - 1));
  *out = limitSize(ents, maxSize);
  return ErrOK;
}

Err TestLogDB::Compact(u64 index) {  // logdb_test.go:159-177
  if (index <= markerIndex) return ErrCompacted;
  if (index > lastIndex()) return ErrUnavailable;
  if (entries.empty()) return ErrUnavailable;
  u64 term;
  Err err = Term(index, &term);
  if (err != ErrOK) return err;
  u64 cut = index - markerIndex;
  entries.erase(entries.begin(), entries.begin() + cut);
  markerIndex = index;
  markerTerm = term;
  return ErrOK;
}

// ---------------------------------------------------------------- inmemory.go
void InMemory::init(u64 lastIndex) {  // inmemory.go:46-57
  markerIndex = lastIndex + 1;
  savedTo = lastIndex;
  newEntries = true;
}

void InMemory::checkMarkerIndex() const {  // inmemory.go:59-66
  if (!entries.empty() && entries[0].index != markerIndex)
    panicf("marker index %llu, first index %llu", (unsigned long long)markerIndex,
           (unsigned long long)entries[0].index);
}

std::vector<Entry> InMemory::getEntries(u64 low, u64 high) const {  // inmemory.go:68-78
  u64 upperBound = markerIndex + entries.size();
  if (low > high || low < markerIndex)
    panicf("invalid low value %llu, high %llu, marker index %llu", (unsigned long long)low,
           (unsigned long long)high, (unsigned long long)markerIndex);
  if (high > upperBound)
    panicf("invalid high value %llu, upperBound %llu", (unsigned long long)high,
           (unsigned long long)upperBound);
  return std::vector<Entry>(entries.begin() + (low - markerIndex),
                            entries.begin() + (high - markerIndex));
}

bool InMemory::getSnapshotIndex(u64* idx) const {  // inmemory.go:80-85
  if (hasSnapshot) {
    *idx = snapshot.index;
    return true;
  }
  *idx = 0;
  return false;
}

bool InMemory::getLastIndex(u64* idx) const {  // inmemory.go:87-92
  if (!entries.empty()) {
    *idx = entries.back().index;
    return true;
  }
  return getSnapshotIndex(idx);
}

bool InMemory::getTerm(u64 index, u64* term) const {  // inmemory.go:94-106
  u64 idx;
  if (index < markerIndex) {
    if (getSnapshotIndex(&idx) && idx == index) {
      *term = snapshot.term;
      return true;
    }
    *term = 0;
    return false;
  }
  bool ok = getLastIndex(&idx);
  if (ok && index <= idx) {
    *term = entries[index - markerIndex].term;
    return true;
  }
  *term = 0;
  return false;
}

void InMemory::commitUpdate(const UpdateCommit& cu) {  // inmemory.go:108-115
  if (cu.stable_log_to > 0) savedLogTo(cu.stable_log_to, cu.stable_log_term);
  if (cu.stable_snapshot_to > 0) savedSnapshotTo(cu.stable_snapshot_to);
}

std::vector<Entry> InMemory::entriesToSave() const {  // inmemory.go:117-123
  u64 idx = savedTo + 1;
  if (idx - markerIndex > (u64)entries.size()) return {};
  return std::vector<Entry>(entries.begin() + (idx - markerIndex), entries.end());
}

void InMemory::savedLogTo(u64 index, u64 term) {  // inmemory.go:125-137
  if (index < markerIndex) return;
  if (entries.empty()) return;
  if (index > entries.back().index || term != entries[index - markerIndex].term) return;
  savedTo = index;
}

void InMemory::appliedLogTo(u64 index) {  // inmemory.go:139-167
  if (index < markerIndex) return;
  if (entries.empty()) return;
  if (index > entries.back().index) return;
  u64 newMarkerIndex = index;
  // applied := entries[:move], less its first entry (the previous marker,
  // already counted off) unless the window was rebuilt since
  u64 move = newMarkerIndex - markerIndex;
  if (newMarkerIndex - markerIndex + 1 <= (u64)entries.size()) move = newMarkerIndex - markerIndex + 1;
  u64 appliedSz = 0;
  if (rateLimited()) {
    std::vector<Entry> applied(entries.begin() + (newEntries ? 0 : 1), entries.begin() + move);
    appliedSz = entrySliceInMemSize(applied);
  }
  newEntries = false;
  shrunk = true;
  entries.erase(entries.begin(), entries.begin() + (newMarkerIndex - markerIndex));
  markerIndex = newMarkerIndex;
  resizeEntrySlice();
  checkMarkerIndex();
  if (rateLimited()) rl->decrease(appliedSz);
}

void InMemory::savedSnapshotTo(u64 index) {  // inmemory.go:169-175
  u64 idx;
  bool ok = getSnapshotIndex(&idx);
  if (ok && idx == index) hasSnapshot = false;
}

void InMemory::resizeEntrySlice() {  // inmemory.go:186-192
  // capacity bookkeeping only; the observable part is the shrunk flag, which
  // resize() clears when the slice is rebuilt.  Go: toResize is true when the
  // free capacity drops below MinEntrySliceFreeSize; a freshly re-sliced slice
  // (the only way shrunk becomes true) is resized when it holds <=1 entry.
  if (shrunk && entries.size() <= 1) resize();
}

void InMemory::merge(const std::vector<Entry>& ents) {  // inmemory.go:201-234
  u64 firstNewIndex = ents[0].index;
  resizeEntrySlice();
  if (firstNewIndex == markerIndex + entries.size()) {
    checkEntriesToAppend(entries, ents);
    entries.insert(entries.end(), ents.begin(), ents.end());
    if (rateLimited()) rl->increase(entrySliceInMemSize(ents));
  } else if (firstNewIndex <= markerIndex) {
    markerIndex = firstNewIndex;
    shrunk = false;
    entries = ents;
    savedTo = firstNewIndex - 1;
    if (rateLimited()) {
      newEntries = true;
      rl->set(entrySliceInMemSize(ents));
    }
  } else {
    std::vector<Entry> existing = getEntries(markerIndex, firstNewIndex);
    checkEntriesToAppend(existing, ents);
    shrunk = false;
    entries = existing;
    entries.insert(entries.end(), ents.begin(), ents.end());
    savedTo = umin(savedTo, firstNewIndex - 1);
    if (rateLimited()) {
      rl->set(entrySliceInMemSize(ents) + entrySliceInMemSize(existing));
      newEntries = true;
    }
  }
  checkMarkerIndex();
}

void InMemory::restore(const Snapshot& ss) {  // inmemory.go:236-246
  snapshot = ss;
  hasSnapshot = true;
  markerIndex = ss.index + 1;
  shrunk = false;
  entries.clear();
  savedTo = ss.index;
  if (rateLimited()) {
    newEntries = true;
    rl->set(0);
  }
}

// ---------------------------------------------------------------- server/rate.go
bool RateLimiter::rateLimited() {  // limitedByInMemSize, rate.go:113-137
  if (!enabled()) return false;
  u64 maxInMemSize = 0;
  bool gcNeeded = false;
  for (auto& kv : followerSizes) {
    if (tick - kv.second.first > RateLimitGcTick) {
      gcNeeded = true;
      continue;
    }
    if (kv.second.second > maxInMemSize) maxInMemSize = kv.second.second;
  }
  u64 sz = get();
  if (sz > maxInMemSize) maxInMemSize = sz;
  if (gcNeeded) gc();
  return maxInMemSize > maxSize;
}

void RateLimiter::gc() {  // rate.go:139-149
  for (auto it = followerSizes.begin(); it != followerSizes.end();) {
    if (tick - it->second.first > RateLimitGcTick) it = followerSizes.erase(it);
    else ++it;
  }
}

u64 entrySliceSize(const std::vector<Entry>& ents) {  // raftpb/raft.go:301-307
  u64 sz = 0;
  for (auto& e : ents) sz += e.sizeUpperLimit();
  return sz;
}

u64 entrySliceInMemSize(const std::vector<Entry>& ents) {  // raftpb/raft.go:311-322
  u64 sz = 0;
  for (auto& e : ents) sz += (u64)e.cmd.size() + GoEntryStructSize;
  return sz;
}

// ---------------------------------------------------------------- logentry.go
void EntryLog::init(ILogDB* db) {  // logentry.go:86-96
  logdb = db;
  auto r = db->GetRange();
  inmem.init(r.second);
  committed = r.first - 1;
  processed = r.first - 1;
}

u64 EntryLog::firstIndex() const {  // logentry.go:98-105
  u64 index;
  if (inmem.getSnapshotIndex(&index)) return index + 1;
  return logdb->GetRange().first;
}

u64 EntryLog::lastIndex() const {  // logentry.go:107-114
  u64 index;
  if (inmem.getLastIndex(&index)) return index;
  return logdb->GetRange().second;
}

std::pair<u64, u64> EntryLog::termEntryRange() const {  // logentry.go:116-125
  return {firstIndex() - 1, lastIndex()};
}

bool EntryLog::entryRange(u64* first, u64* last) const {  // logentry.go:127-132
  if (inmem.hasSnapshot && inmem.entries.empty()) return false;
  *first = firstIndex();
  *last = lastIndex();
  return true;
}

u64 EntryLog::lastTerm() const {  // logentry.go:134-140
  u64 t;
  Err err = term(lastIndex(), &t);
  if (err != ErrOK) panicf("lastTerm: %d", err);
  return t;
}

Err EntryLog::term(u64 index, u64* t) const {  // logentry.go:142-161
  auto r = termEntryRange();
  if (index < r.first || index > r.second) {
    *t = 0;
    return ErrOK;
  }
  if (inmem.getTerm(index, t)) return ErrOK;
  Err err = logdb->Term(index, t);
  if (err != ErrOK && err != ErrCompacted && err != ErrUnavailable) panicf("term err %d", err);
  if (err == ErrOK) return ErrOK;
  *t = 0;
  return err;
}

Err EntryLog::checkBound(u64 low, u64 high) const {  // logentry.go:163-178
  if (low > high) panicf("input low %llu > high %llu", (unsigned long long)low, (unsigned long long)high);
  u64 first, last;
  if (!entryRange(&first, &last)) return ErrCompacted;
  if (low < first) return ErrCompacted;
  if (high > last + 1)
    panicf("requested range [%llu,%llu) is out of bound [%llu,%llu]", (unsigned long long)low,
           (unsigned long long)high, (unsigned long long)first, (unsigned long long)last);
  return ErrOK;
}

std::vector<Entry> EntryLog::getUncommittedEntries() const {  // logentry.go:180-183
  u64 li = inmem.markerIndex + inmem.entries.size();
  return getEntriesFromInMem({}, committed + 1, li);
}

Err EntryLog::getEntriesFromLogDB(u64 low, u64 high, u64 maxSize, std::vector<Entry>* ents,
                                  bool* checkInMem) const {  // logentry.go:185-203
  ents->clear();
  if (low >= inmem.markerIndex) {
    *checkInMem = true;
    return ErrOK;
  }
  u64 upperBound = umin(high, inmem.markerIndex);
  Err err = logdb->Entries(low, upperBound, maxSize, ents);
  if (err == ErrCompacted) {
    *checkInMem = false;
    return err;
  } else if (err != ErrOK) {
    panicf("getEntriesFromLogDB err %d", err);
  }
  if ((u64)ents->size() > upperBound - low) panicf("uint64(len(ents)) > upperBound-low");
  *checkInMem = (u64)ents->size() == upperBound - low;
  return ErrOK;
}

std::vector<Entry> EntryLog::getEntriesFromInMem(std::vector<Entry> ents, u64 low,
                                                 u64 high) const {  // logentry.go:205-220
  if (high <= inmem.markerIndex) return ents;
  u64 lowerBound = umax(low, inmem.markerIndex);
  std::vector<Entry> im = inmem.getEntries(lowerBound, high);
  if (!im.empty()) {
    if (!ents.empty()) {
      checkEntriesToAppend(ents, im);
      ents.insert(ents.end(), im.begin(), im.end());
      return ents;
    }
    return im;
  }
  return ents;
}

Err EntryLog::getEntries(u64 low, u64 high, u64 maxSize,
                         std::vector<Entry>* out) const {  // logentry.go:222-239
  out->clear();
  Err err = checkBound(low, high);
  if (err != ErrOK) return err;
  if (low == high) return ErrOK;
  std::vector<Entry> ents;
  bool checkInMem = false;
  err = getEntriesFromLogDB(low, high, maxSize, &ents, &checkInMem);
  if (err != ErrOK) return err;
  if (!checkInMem) {
    *out = ents;
    return ErrOK;
  }
  *out = limitSize(getEntriesFromInMem(ents, low, high), maxSize);
  return ErrOK;
}

Err EntryLog::entries(u64 start, u64 maxSize, std::vector<Entry>* out) const {  // logentry.go:241-246
  out->clear();
  if (start > lastIndex()) return ErrOK;
  return getEntries(start, lastIndex() + 1, maxSize, out);
}

Snapshot EntryLog::snapshot() const {  // logentry.go:248-253
  if (inmem.hasSnapshot) return inmem.snapshot;
  return logdb->GetSnapshot();
}

u64 EntryLog::firstNotAppliedIndex() const {  // logentry.go:255-257
  return umax(processed + 1, firstIndex());
}

bool EntryLog::hasEntriesToApply() const {  // logentry.go:263-265
  return toApplyIndexLimit() > firstNotAppliedIndex();
}

std::vector<Entry> EntryLog::getEntriesToApply(u64 limit) const {  // logentry.go:275-285
  if (hasEntriesToApply()) {
    std::vector<Entry> ents;
    Err err = getEntries(firstNotAppliedIndex(), toApplyIndexLimit(), limit, &ents);
    if (err != ErrOK) panicf("getEntriesToApply err %d", err);
    return ents;
  }
  return {};
}

bool EntryLog::tryAppend(u64 index, const std::vector<Entry>& ents) {  // logentry.go:291-302
  u64 conflictIndex = getConflictIndex(ents);
  if (conflictIndex != 0) {
    if (conflictIndex <= committed)
      panicf("entry %llu conflicts with committed entry, committed %llu",
             (unsigned long long)conflictIndex, (unsigned long long)committed);
    append(std::vector<Entry>(ents.begin() + (conflictIndex - index - 1), ents.end()));
    return true;
  }
  return false;
}

void EntryLog::append(const std::vector<Entry>& entries) {  // logentry.go:304-313
  if (entries.empty()) return;
  if (entries[0].index <= committed)
    panicf("committed entries being changed, committed %llu, first idx %llu",
           (unsigned long long)committed, (unsigned long long)entries[0].index);
  inmem.merge(entries);
}

u64 EntryLog::getConflictIndex(const std::vector<Entry>& entries) const {  // logentry.go:315-322
  for (auto& e : entries)
    if (!matchTerm(e.index, e.term)) return e.index;
  return 0;
}

void EntryLog::commitTo(u64 index) {  // logentry.go:324-333
  if (index <= committed) return;
  if (index > lastIndex())
    panicf("invalid commitTo index %llu, lastIndex() %llu", (unsigned long long)index,
           (unsigned long long)lastIndex());
  committed = index;
}

void EntryLog::commitUpdate(const UpdateCommit& cu) {  // logentry.go:335-355
  inmem.commitUpdate(cu);
  if (cu.processed > 0) {
    if (cu.processed < processed || cu.processed > committed)
      panicf("invalid ApplyReturnedTo %llu, current applied %llu, committed %llu",
             (unsigned long long)cu.processed, (unsigned long long)processed,
             (unsigned long long)committed);
    processed = cu.processed;
  }
  if (cu.last_applied > 0) {
    if (cu.last_applied > committed) panicf("invalid last applied");
    if (cu.last_applied > processed) panicf("invalid last applied vs processed");
    inmem.appliedLogTo(cu.last_applied);
  }
}

bool EntryLog::matchTerm(u64 index, u64 t) const {  // logentry.go:357-363
  u64 lt;
  if (term(index, &lt) != ErrOK) return false;
  return lt == t;
}

bool EntryLog::upToDate(u64 index, u64 t) const {  // logentry.go:365-377
  u64 lt;
  if (term(lastIndex(), &lt) != ErrOK) panicf("failed to get the last term");
  if (t >= lt) {
    if (t > lt) return true;
    return index >= lastIndex();
  }
  return false;
}

bool EntryLog::tryCommit(u64 index, u64 t) {  // logentry.go:379-394
  if (index <= committed) return false;
  u64 lterm;
  Err err = term(index, &lterm);
  if (err == ErrCompacted) lterm = 0;
  else if (err != ErrOK) panicf("tryCommit term err %d", err);
  if (index > committed && lterm == t) {
    commitTo(index);
    return true;
  }
  return false;
}

void EntryLog::restore(const Snapshot& s) {  // logentry.go:396-401
  inmem.restore(s);
  committed = s.index;
  processed = s.index;
}

// ---------------------------------------------------------------- remote.go
void Remote::becomeRetry() {  // remote.go:75-83
  if (state == RemoteSnapshot) next = umax(match + 1, snapshotIndex + 1);
  else next = match + 1;
  reset();
  state = RemoteRetry;
}

void Remote::becomeReplicate() {  // remote.go:102-106
  next = match + 1;
  reset();
  state = RemoteReplicate;
}

void Remote::becomeSnapshot(u64 index) {  // remote.go:108-112
  reset();
  snapshotIndex = index;
  state = RemoteSnapshot;
}

bool Remote::tryUpdate(u64 index) {  // remote.go:123-133
  if (next < index + 1) next = index + 1;
  if (match < index) {
    waitToRetry();
    match = index;
    return true;
  }
  return false;
}

void Remote::progress(u64 lastIndex) {  // remote.go:135-143
  if (state == RemoteReplicate) next = lastIndex + 1;
  else if (state == RemoteRetry) retryToWait();
  else panicf("unexpected remote state");
}

void Remote::respondedTo() {  // remote.go:145-153
  if (state == RemoteRetry) becomeReplicate();
  else if (state == RemoteSnapshot) {
    if (match >= snapshotIndex) becomeRetry();
  }
}

bool Remote::decreaseTo(u64 rejected, u64 last) {  // remote.go:155-171
  if (state == RemoteReplicate) {
    if (rejected <= match) return false;
    next = match + 1;
    return true;
  }
  if (next - 1 != rejected) return false;
  waitToRetry();
  next = umax(1, umin(rejected, last + 1));
  return true;
}

bool Remote::isPaused() const {  // remote.go:173-186
  switch (state) {
    case RemoteRetry: return false;
    case RemoteWait: return true;
    case RemoteReplicate: return false;
    case RemoteSnapshot: return true;
    default: panicf("unexpected remote state");
  }
}

// ---------------------------------------------------------------- readindex.go
void ReadIndexQ::addRequest(u64 index, SystemCtx ctx, u64 from) {  // readindex.go:43-67
  if (pending.count(ctx)) return;
  if (!queue.empty()) {
    auto it = pending.find(peepCtx());
    if (it == pending.end()) panicf("inconsistent pending and queue");
    if (index < it->second.index) panicf("index moved backward in readIndex");
  }
  queue.push_back(ctx);
  ReadStatus s;
  s.index = index;
  s.from = from;
  s.ctx = ctx;
  pending[ctx] = s;
}

std::vector<ReadStatus> ReadIndexQ::confirm(SystemCtx ctx, u64 from,
                                            int quorum) {  // readindex.go:77-116
  auto it = pending.find(ctx);
  if (it == pending.end()) return {};
  it->second.confirmed.insert(from);
  if ((int)it->second.confirmed.size() + 1 < quorum) return {};
  size_t done = 0;
  std::vector<ReadStatus> cs;
  for (auto& pctx : queue) {
    done++;
    auto sit = pending.find(pctx);
    if (sit == pending.end()) panicf("inconsistent pending and queue content");
    cs.push_back(sit->second);
    if (pctx == ctx) {
      u64 sindex = sit->second.index;
      for (auto& v : cs) {
        if (v.index > sindex) panicf("v.index > s.index is unexpected");
        v.index = sindex;
      }
      queue.erase(queue.begin(), queue.begin() + done);
      for (auto& v : cs) pending.erase(v.ctx);
      if (queue.size() != pending.size()) panicf("inconsistent length");
      return cs;
    }
  }
  return {};
}

// ---------------------------------------------------------------- raft.go
Raft::Raft(const Config& c, ILogDB* logdb) {  // newRaft, raft.go:234-289
  if (c.nodeID == 0) panicf("invalid node id");
  if (c.electionRTT == 0 || c.heartbeatRTT == 0 || c.electionRTT <= 2 * c.heartbeatRTT)
    panicf("invalid election/heartbeat rtt");  // config.go Validate
  if (logdb == nullptr) panicf("logdb is nil");
  rl.maxSize = c.maxInMemLogSize;  // server.NewRateLimiter(c.MaxInMemLogSize)
  log.inmem.rl = &rl;
  clusterID = c.clusterID;
  nodeID = c.nodeID;
  leaderID = NoLeader;
  log.maxEntrySize = c.maxEntrySize;
  maxEntrySize = c.maxEntrySize;
  log.init(logdb);
  electionTimeout = c.electionRTT;
  heartbeatTimeout = c.heartbeatRTT;
  checkQuorum = c.checkQuorum;
  rngSeed = c.rngSeed;
  auto ns = logdb->NodeState();
  for (auto& p : ns.second.addresses) remotes[p.first] = Remote{0, 1};
  for (auto& p : ns.second.observers) observers[p.first] = Remote{0, 1};
  for (auto& p : ns.second.witnesses) witnesses[p.first] = Remote{0, 1};
  resetMatchValueArray();
  if (!isEmptyState(ns.first)) loadState(ns.first);
  if (c.isObserver) {
    state = Observer;
    becomeObserver(term, NoLeader);
  } else if (c.isWitness) {
    state = Witness;
    becomeWitness(term, NoLeader);
  } else {
    becomeFollower(term, NoLeader);
  }
}

void Raft::setTestPeers(const std::vector<u64>& peers) {  // raft.go:291-297
  if (remotes.empty())
    for (u64 p : peers) remotes[p] = Remote{0, 1};
}

void Raft::mustBeLeader() const {  // raft.go:339-343
  if (!isLeader()) panicf("%llu is not a leader", (unsigned long long)nodeID);
}

void Raft::setLeaderID(u64 id) {  // raft.go:345-356
  leaderID = id;
  if (hasEvents) events.leaderUpdated++;
}

bool Raft::leaderHasQuorum() {  // raft.go:378-388
  int c = 0;
  for (auto& kv : votingMembers()) {
    if (kv.first == nodeID || kv.second->isActive()) {
      c++;
      kv.second->setNotActive();
    }
  }
  return c >= quorum();
}

std::vector<u64> Raft::nodes() const {  // raft.go:390-402
  std::vector<u64> out;
  for (auto& kv : remotes) out.push_back(kv.first);
  for (auto& kv : observers) out.push_back(kv.first);
  for (auto& kv : witnesses) out.push_back(kv.first);
  return out;
}

std::vector<u64> Raft::nodesSorted() const {  // raft.go:404-408
  auto n = nodes();
  std::sort(n.begin(), n.end());
  return n;
}

std::map<u64, Remote*> Raft::votingMembers() {  // raft.go:410-419
  std::map<u64, Remote*> out;
  for (auto& kv : remotes) out[kv.first] = &kv.second;
  for (auto& kv : witnesses) out[kv.first] = &kv.second;
  return out;
}

void Raft::loadState(const PState& st) {  // raft.go:429-437
  if (st.commit < log.committed || st.commit > log.lastIndex())
    panicf("got out of range state, st.commit %llu, range[%llu,%llu]",
           (unsigned long long)st.commit, (unsigned long long)log.committed,
           (unsigned long long)log.lastIndex());
  log.committed = st.commit;
  term = st.term;
  vote = st.vote;
}

bool Raft::restore(const Snapshot& ss) {  // raft.go:439-470
  if (ss.index <= log.committed) return false;
  if (!isObserver())
    for (auto& kv : ss.membership.observers)
      if (kv.first == nodeID) panicf("converting to observer");
  if (!isWitness())
    for (auto& kv : ss.membership.witnesses)
      if (kv.first == nodeID) panicf("converting to witness");
  if (log.matchTerm(ss.index, ss.term)) {
    log.commitTo(ss.index);
    return false;
  }
  log.restore(ss);
  return true;
}

void Raft::restoreRemotes(const Snapshot& ss) {  // raft.go:472-517
  remotes.clear();
  for (auto& kv : ss.membership.addresses) {
    u64 id = kv.first;
    if (id == nodeID && isObserver()) becomeFollower(term, leaderID);
    if (witnesses.count(id)) panicf("Assumed witness could not promote to full member");
    u64 match = 0, next = log.lastIndex() + 1;
    if (id == nodeID) match = next - 1;
    setRemote(id, match, next);
  }
  if (selfRemoved() && isLeader()) becomeFollower(term, NoLeader);
  observers.clear();
  for (auto& kv : ss.membership.observers) {
    u64 id = kv.first;
    u64 match = 0, next = log.lastIndex() + 1;
    if (id == nodeID) match = next - 1;
    setObserver(id, match, next);
  }
  witnesses.clear();
  for (auto& kv : ss.membership.witnesses) {
    u64 id = kv.first;
    u64 match = 0, next = log.lastIndex() + 1;
    if (id == nodeID) match = next - 1;
    setWitness(id, match, next);
  }
  resetMatchValueArray();
}

void Raft::tick() {  // raft.go:551-564
  quiesce = false;
  tickCount++;
  if (timeForInMemGC()) log.inmem.tryResize();
  if (isLeader()) leaderTick();
  else nonLeaderTick();
}

void Raft::nonLeaderTick() {  // raft.go:566-590
  if (isLeader()) panicf("noleader tick called on leader node");
  electionTick++;
  if (timeForRateLimitCheck() && rl.enabled()) {
    rl.heartbeatTick();
    sendRateLimitMessage();
  }
  if (isObserver() || isWitness()) return;
  if (!selfRemoved() && timeForElection()) {
    electionTick = 0;
    Message m;
    m.from = nodeID;
    m.type = Election;
    Handle(m);
  }
}

void Raft::leaderTick() {  // raft.go:592-621
  mustBeLeader();
  electionTick++;
  if (timeForRateLimitCheck() && rl.enabled()) rl.heartbeatTick();
  bool abortLT = timeToAbortLeaderTransfer();
  if (timeForCheckQuorum()) {
    electionTick = 0;
    if (checkQuorum) {
      Message m;
      m.from = nodeID;
      m.type = CheckQuorum;
      Handle(m);
    }
  }
  if (abortLT) abortLeaderTransfer();
  heartbeatTick++;
  if (timeForHearbeat()) {
    heartbeatTick = 0;
    Message m;
    m.from = nodeID;
    m.type = LeaderHeartbeat;
    Handle(m);
  }
}

void Raft::quiescedTick() {  // raft.go:623-629
  if (!quiesce) {
    quiesce = true;
    log.inmem.resize();
  }
  electionTick++;
}

void Raft::setRandomizedElectionTimeout() {  // raft.go:631-634
  u64 randTime = below(rto_rand(rngSeed, clusterID, nodeID, rngCount++), electionTimeout);
  randomizedElectionTimeout = electionTimeout + randTime;
}

Message Raft::finalizeMessageTerm(Message m) const {  // raft.go:640-652
  if (m.term == 0 && m.type == RequestVote) panicf("sending RequestVote with 0 term");
  if (m.term > 0 && m.type != RequestVote) panicf("term unexpectedly set for message type %d", m.type);
  if (!(m.type == Propose || m.type == ReadIndex)) m.term = term;
  return m;
}

void Raft::send(Message m) {  // raft.go:654-658
  m.from = nodeID;
  m = finalizeMessageTerm(m);
  msgs.push_back(std::move(m));
}

void Raft::makeInstallSnapshotMessage(u64 to, Message* m, u64* index) {  // raft.go:684-697
  m->to = to;
  m->type = InstallSnapshot;
  Snapshot ss = log.snapshot();
  if (isEmptySnapshot(ss)) panicf("got an empty snapshot");
  if (witnesses.count(to)) {  // makeWitnessSnapshot, raft.go:699-707
    ss.filepath = "";
    ss.file_size = 0;
    ss.files = 0;
    ss.witness = true;
    ss.dummy = false;
  }
  m->snapshot = ss;
  *index = ss.index;
}

Err Raft::makeReplicateMessage(u64 to, u64 next, u64 maxSize, Message* out) {  // raft.go:709-740
  u64 t;
  Err err = log.term(next - 1, &t);
  if (err != ErrOK) return err;
  std::vector<Entry> ents;
  err = log.entries(next, maxSize, &ents);
  if (err != ErrOK) return err;
  if (!ents.empty()) {
    u64 lastIndex = ents.back().index;
    u64 expected = next - 1 + ents.size();
    if (lastIndex != expected) panicf("expected last index in Replicate %llu, got %llu",
                                      (unsigned long long)expected, (unsigned long long)lastIndex);
  }
  if (witnesses.count(to)) {  // makeMetadataEntries, raft.go:742-756
    std::vector<Entry> me;
    for (auto& e : ents) {
      if (e.type != ConfigChangeEntry) {
        Entry x;
        x.type = MetadataEntry;
        x.index = e.index;
        x.term = e.term;
        me.push_back(x);
      } else {
        me.push_back(e);
      }
    }
    ents = me;
  }
  Message m;
  m.to = to;
  m.type = Replicate;
  m.log_index = next - 1;
  m.log_term = t;
  m.entries = std::move(ents);
  m.commit = log.committed;
  *out = std::move(m);
  return ErrOK;
}

void Raft::sendReplicateMessage(u64 to) {  // raft.go:758-792
  Remote* rp = nullptr;
  auto a = remotes.find(to);
  if (a != remotes.end()) rp = &a->second;
  else {
    auto b = observers.find(to);
    if (b != observers.end()) rp = &b->second;
    else {
      auto c = witnesses.find(to);
      if (c == witnesses.end()) panicf("failed to get the remote instance");
      rp = &c->second;
    }
  }
  if (rp->isPaused()) return;
  Message m;
  Err err = makeReplicateMessage(to, rp->next, maxEntrySize, &m);
  if (err != ErrOK) {
    if (!rp->isActive()) return;
    u64 index;
    m = Message();
    makeInstallSnapshotMessage(to, &m, &index);
    rp->becomeSnapshot(index);
  } else {
    if (!m.entries.empty()) rp->progress(m.entries.back().index);
  }
  send(std::move(m));
}

void Raft::broadcastReplicateMessage() {  // raft.go:794-808
  if (!isLeader()) panicf("non-leader broadcasting replication msg");
  for (auto& kv : observers)
    if (kv.first == nodeID) panicf("observer is broadcasting Replicate msg");
  for (u64 nid : nodes())
    if (nid != nodeID) sendReplicateMessage(nid);
}

void Raft::sendHeartbeatMessage(u64 to, SystemCtx hint, u64 match) {  // raft.go:810-820
  Message m;
  m.to = to;
  m.type = Heartbeat;
  m.commit = umin(match, log.committed);
  m.hint = hint.low;
  m.hint_high = hint.high;
  send(std::move(m));
}

void Raft::broadcastHeartbeatMessage() {  // raft.go:824-832
  mustBeLeader();
  if (readIndex.hasPendingRequest()) broadcastHeartbeatMessageWithHint(readIndex.peepCtx());
  else broadcastHeartbeatMessageWithHint(SystemCtx{});
}

void Raft::broadcastHeartbeatMessageWithHint(SystemCtx ctx) {  // raft.go:834-846
  SystemCtx zero;
  for (auto& kv : votingMembers())
    if (kv.first != nodeID) sendHeartbeatMessage(kv.first, ctx, kv.second->match);
  if (ctx == zero)
    for (auto& kv : observers) sendHeartbeatMessage(kv.first, zero, kv.second.match);
}

void Raft::sendTimeoutNowMessage(u64 id) {  // raft.go:848-853
  Message m;
  m.type = TimeoutNow;
  m.to = id;
  send(std::move(m));
}

void Raft::sortMatchValues() {  // raft.go:859-884
  std::sort(matched.begin(), matched.end());
}

bool Raft::tryCommit() {  // raft.go:886-907
  mustBeLeader();
  if (numVotingMembers() != matched.size()) resetMatchValueArray();
  size_t idx = 0;
  for (auto& kv : remotes) matched[idx++] = kv.second.match;
  for (auto& kv : witnesses) matched[idx++] = kv.second.match;
  sortMatchValues();
  u64 q = matched[numVotingMembers() - quorum()];
  return log.tryCommit(q, term);
}

void Raft::appendEntries(std::vector<Entry> entries) {  // raft.go:909-920
  u64 lastIndex = log.lastIndex();
  for (size_t i = 0; i < entries.size(); i++) {
    entries[i].term = term;
    entries[i].index = lastIndex + 1 + i;
  }
  log.append(entries);
  auto self = remotes.find(nodeID);
  if (self == remotes.end()) panicf("nil remote for self");  // Go: nil map value deref
  self->second.tryUpdate(log.lastIndex());
  if (isSingleNodeQuorum()) tryCommit();
}

void Raft::becomeObserver(u64 t, u64 lid) {  // raft.go:926-936
  if (!isObserver()) panicf("transitioning to observer state from non-observer");
  reset(t);
  setLeaderID(lid);
}

void Raft::becomeWitness(u64 t, u64 lid) {  // raft.go:938-945
  if (!isWitness()) panicf("transitioning to witness state from non-witness");
  reset(t);
  setLeaderID(lid);
}

void Raft::becomeFollower(u64 t, u64 lid) {  // raft.go:947-955
  if (isWitness()) panicf("transitioning to follower from witness state");
  state = Follower;
  reset(t);
  setLeaderID(lid);
}

void Raft::becomeCandidate() {  // raft.go:957-973
  if (isLeader()) panicf("transitioning to candidate state from leader");
  if (isObserver()) panicf("observer is becoming candidate");
  if (isWitness()) panicf("witness is becoming candidate");
  state = Candidate;
  reset(term + 1);
  setLeaderID(NoLeader);
  vote = nodeID;
}

void Raft::becomeLeader() {  // raft.go:975-987
  if (!isLeader() && !isCandidate()) panicf("transitioning to leader state from %d", state);
  state = Leader;
  reset(term);
  setLeaderID(nodeID);
  preLeaderPromotionHandleConfigChange();
  std::vector<Entry> ents(1);
  ents[0].type = ApplicationEntry;
  appendEntries(ents);
}

void Raft::reset(u64 t) {  // raft.go:989-1008
  if (term != t) {
    term = t;
    vote = NoLeader;
  }
  if (rl.enabled()) rl.resetFollowerState();
  votes.clear();
  electionTick = 0;
  heartbeatTick = 0;
  setRandomizedElectionTimeout();
  readIndex = ReadIndexQ();
  pendingConfigChange = false;
  abortLeaderTransfer();
  resetRemotes();
  resetObservers();
  resetWitnesses();
  resetMatchValueArray();
}

void Raft::preLeaderPromotionHandleConfigChange() {  // raft.go:1010-1018
  int n = getPendingConfigChangeCount();
  if (n > 1) panicf("multiple uncommitted config change entries");
  else if (n == 1) pendingConfigChange = true;
}

void Raft::resetRemotes() {  // raft.go:1023-1032
  for (auto& kv : remotes) {
    kv.second = Remote{0, log.lastIndex() + 1};
    if (kv.first == nodeID) kv.second.match = log.lastIndex();
  }
}

void Raft::resetObservers() {  // raft.go:1034-1043
  for (auto& kv : observers) {
    kv.second = Remote{0, log.lastIndex() + 1};
    if (kv.first == nodeID) kv.second.match = log.lastIndex();
  }
}

void Raft::resetWitnesses() {  // raft.go:1045-1054
  for (auto& kv : witnesses) {
    kv.second = Remote{0, log.lastIndex() + 1};
    if (kv.first == nodeID) kv.second.match = log.lastIndex();
  }
}

int Raft::handleVoteResp(u64 from, bool rejected) {  // raft.go:1060-1078
  int votedFor = 0;
  if (!votes.count(from)) votes[from] = !rejected;
  for (auto& kv : votes)
    if (kv.second) votedFor++;
  return votedFor;
}

void Raft::campaign() {  // raft.go:1080-1116
  becomeCandidate();
  u64 t = term;
  if (hasEvents) events.campaignLaunched++;
  handleVoteResp(nodeID, false);
  if (isSingleNodeQuorum()) {
    becomeLeader();
    return;
  }
  u64 hint = 0;
  if (isLeaderTransferTarget) {
    hint = nodeID;
    isLeaderTransferTarget = false;
  }
  for (auto& kv : votingMembers()) {
    if (kv.first == nodeID) continue;
    Message m;
    m.term = t;
    m.to = kv.first;
    m.type = RequestVote;
    m.log_index = log.lastIndex();
    m.log_term = log.lastTerm();
    m.hint = hint;
    send(std::move(m));
  }
}

bool Raft::selfRemoved() const {  // raft.go:1122-1133
  if (isObserver()) return !observers.count(nodeID);
  if (isWitness()) return !witnesses.count(nodeID);
  return !remotes.count(nodeID);
}

void Raft::addNode(u64 id) {  // raft.go:1135-1157
  pendingConfigChange = false;
  if (id == nodeID && isWitness()) panicf("is a witness");
  if (remotes.count(id)) return;
  auto it = observers.find(id);
  if (it != observers.end()) {
    Remote rp = it->second;
    observers.erase(it);
    remotes[id] = rp;
    if (id == nodeID) becomeFollower(term, leaderID);
  } else if (witnesses.count(id)) {
    panicf("could not promote witness to a full member");
  } else {
    setRemote(id, 0, log.lastIndex() + 1);
  }
}

void Raft::addObserver(u64 id) {  // raft.go:1159-1168
  pendingConfigChange = false;
  if (id == nodeID && !isObserver()) panicf("is not an observer");
  if (observers.count(id)) return;
  setObserver(id, 0, log.lastIndex() + 1);
}

void Raft::addWitness(u64 id) {  // raft.go:1170-1179
  pendingConfigChange = false;
  if (id == nodeID && !isWitness()) panicf("is not a witness");
  if (witnesses.count(id)) return;
  setWitness(id, 0, log.lastIndex() + 1);
}

void Raft::removeNode(u64 id) {  // raft.go:1181-1198
  remotes.erase(id);
  observers.erase(id);
  witnesses.erase(id);
  pendingConfigChange = false;
  if (nodeID == id && isLeader()) becomeFollower(term, NoLeader);
  if (leaderTransfering() && leaderTransferTarget == id) abortLeaderTransfer();
  if (isLeader() && numVotingMembers() > 0) {
    if (tryCommit()) broadcastReplicateMessage();
  }
}

void Raft::setRemote(u64 id, u64 match, u64 next) {  // raft.go:1212-1219
  Remote r;
  r.next = next;
  r.match = match;
  remotes[id] = r;
}

void Raft::setObserver(u64 id, u64 match, u64 next) {  // raft.go:1221-1228
  Remote r;
  r.next = next;
  r.match = match;
  observers[id] = r;
}

void Raft::setWitness(u64 id, u64 match, u64 next) {  // raft.go:1230-1237
  Remote r;
  r.next = next;
  r.match = match;
  witnesses[id] = r;
}

int Raft::getPendingConfigChangeCount() {  // raft.go:1281-1295
  u64 idx = log.committed + 1;
  int count = 0;
  for (;;) {
    std::vector<Entry> ents;
    Err err = log.entries(idx, maxEntrySize, &ents);
    if (err != ErrOK) panicf("failed to get entries %d", err);
    if (ents.empty()) return count;
    count += countConfigChange(ents);
    idx = ents.back().index + 1;
  }
}

void Raft::handleHeartbeatMessage(const Message& m) {  // raft.go:1301-1309
  log.commitTo(m.commit);
  Message r;
  r.to = m.from;
  r.type = HeartbeatResp;
  r.hint = m.hint;
  r.hint_high = m.hint_high;
  send(std::move(r));
}

void Raft::handleInstallSnapshotMessage(const Message& m) {  // raft.go:1311-1337
  Message resp;
  resp.to = m.from;
  resp.type = ReplicateResp;
  if (restore(m.snapshot)) {
    resp.log_index = log.lastIndex();
  } else {
    resp.log_index = log.committed;
    if (hasEvents) events.snapshotRejected++;
  }
  send(std::move(resp));
}

void Raft::handleReplicateMessage(const Message& m) {  // raft.go:1339-1372
  Message resp;
  resp.to = m.from;
  resp.type = ReplicateResp;
  if (m.log_index < log.committed) {
    resp.log_index = log.committed;
    send(std::move(resp));
    return;
  }
  if (log.matchTerm(m.log_index, m.log_term)) {
    log.tryAppend(m.log_index, m.entries);
    u64 lastIdx = m.log_index + m.entries.size();
    log.commitTo(umin(lastIdx, m.commit));
    resp.log_index = lastIdx;
  } else {
    resp.reject = true;
    resp.log_index = m.log_index;
    resp.hint = log.lastIndex();
    if (hasEvents) events.replicationRejected++;
  }
  send(std::move(resp));
}

static bool isLeaderMessage(int t) {  // raft.go:1382-1385
  return t == Replicate || t == InstallSnapshot || t == Heartbeat || t == TimeoutNow ||
         t == ReadIndexResp;
}

bool Raft::dropRequestVoteFromHighTermNode(const Message& m) {  // raft.go:1387-1409
  if (m.type != RequestVote || !checkQuorum || m.term <= term) return false;
  if (m.hint == m.from) return false;
  if (isLeader() && !quiesce && electionTick >= electionTimeout)
    panicf("r.electionTick >= r.electionTimeout on leader");
  if (leaderID != NoLeader && electionTick < electionTimeout) return true;
  return false;
}

bool Raft::onMessageTermNotMatched(const Message& m) {  // raft.go:1415-1449
  if (m.term == 0 || m.term == term) return false;
  if (dropRequestVoteFromHighTermNode(m)) return true;
  if (m.term > term) {
    u64 lid = NoLeader;
    if (isLeaderMessage(m.type)) lid = m.from;
    if (isObserver()) becomeObserver(m.term, lid);
    else if (isWitness()) becomeWitness(m.term, lid);
    else becomeFollower(m.term, lid);
  } else if (m.term < term) {
    if (isLeaderMessage(m.type) && checkQuorum) {
      Message r;
      r.to = m.from;
      r.type = NoOP;
      send(std::move(r));
    }
    return true;
  }
  return false;
}

void Raft::doubleCheckTermMatched(u64 msgTerm) const {  // raft.go:1922-1926
  if (msgTerm != 0 && term != msgTerm) panicf("mismatched term found");
}

void Raft::Handle(Message m) {  // raft.go:1451-1458
  if (!onMessageTermNotMatched(m)) {
    doubleCheckTermMatched(m.term);
    dispatch(m);
  }
}

bool Raft::testOnlyHasConfigChangeToApply() {  // raft_etcd_test.go:47-54
  std::vector<Entry> ents = log.getEntriesToApply(NoLimit);
  if (log.committed > log.processed && !ents.empty()) return countConfigChange(ents) > 0;
  return false;
}

bool Raft::hasConfigChangeToApply() {  // raft.go:1460-1472
  if (testOnlyCCMode) return testOnlyHasConfigChangeToApply();
  return log.committed > applied;
}

void Raft::handleNodeElection(const Message&) {  // raft.go:1482-1512
  if (!isLeader()) {
    if (hasConfigChangeToApply()) {
      if (hasEvents) events.campaignSkipped++;
      return;
    }
    campaign();
  }
}

void Raft::handleNodeRequestVote(const Message& m) {  // raft.go:1514-1535
  Message resp;
  resp.to = m.from;
  resp.type = RequestVoteResp;
  bool canGrant = canGrantVote(m);
  bool isUpToDate = log.upToDate(m.log_index, m.log_term);
  if (canGrant && isUpToDate) {
    electionTick = 0;
    vote = m.from;
  } else {
    resp.reject = true;
  }
  send(std::move(resp));
}

void Raft::handleNodeConfigChange(const Message& m) {  // raft.go:1537-1556
  if (m.reject) {
    pendingConfigChange = false;
  } else {
    int cctype = (int)m.hint_high;
    u64 nid = m.hint;
    switch (cctype) {
      case AddNode: addNode(nid); break;
      case RemoveNode: removeNode(nid); break;
      case AddObserver: addObserver(nid); break;
      case AddWitness: addWitness(nid); break;
      default: panicf("unexpected config change type");
    }
  }
}

void Raft::handleLocalTick(const Message& m) {  // raft.go:1558-1564
  if (m.reject) quiescedTick();
  else tick();
}

void Raft::handleRestoreRemote(const Message& m) { restoreRemotes(m.snapshot); }  // raft.go:1566-1568

void Raft::handleLeaderHeartbeat(const Message&) { broadcastHeartbeatMessage(); }  // raft.go:1574-1576

void Raft::handleLeaderCheckQuorum(const Message&) {  // raft.go:1579-1585
  mustBeLeader();
  if (!leaderHasQuorum()) becomeFollower(term, NoLeader);
}

void Raft::handleLeaderPropose(Message& m) {  // raft.go:1587-1606
  mustBeLeader();
  if (leaderTransfering()) {
    reportDroppedProposal(m);
    return;
  }
  for (size_t i = 0; i < m.entries.size(); i++) {
    if (m.entries[i].type == ConfigChangeEntry) {
      if (pendingConfigChange) {
        reportDroppedConfigChange(m.entries[i]);
        m.entries[i] = Entry();
        m.entries[i].type = ApplicationEntry;
      }
      pendingConfigChange = true;
    }
  }
  appendEntries(m.entries);
  broadcastReplicateMessage();
}

bool Raft::hasCommittedEntryAtCurrentTerm() const {  // raft.go:1609-1618
  if (term == 0) panicf("not suppose to reach here");
  u64 lct;
  Err err = log.term(log.committed, &lct);
  if (err != ErrOK && err != ErrCompacted) panicf("failed to get term");
  return lct == term;
}

void Raft::handleLeaderReadIndex(const Message& m) {  // raft.go:1633-1665
  mustBeLeader();
  SystemCtx ctx{m.hint, m.hint_high};
  if (!isSingleNodeQuorum()) {
    if (!hasCommittedEntryAtCurrentTerm()) {
      reportDroppedReadIndex(m);
      return;
    }
    readIndex.addRequest(log.committed, ctx, m.from);
    broadcastHeartbeatMessageWithHint(ctx);
  } else {
    addReadyToRead(log.committed, ctx);
    bool ook = observers.count(m.from) > 0;
    bool wok = witnesses.count(m.from) > 0;
    if (m.from != nodeID && (ook || wok)) {
      Message r;
      r.to = m.from;
      r.type = ReadIndexResp;
      r.log_index = log.committed;
      r.hint = m.hint;
      r.hint_high = m.hint_high;
      r.commit = m.commit;
      send(std::move(r));
    }
  }
}

void Raft::handleLeaderReplicateResp(const Message& m, Remote* rp) {  // raft.go:1667-1696
  mustBeLeader();
  rp->setActive();
  if (!m.reject) {
    bool paused = rp->isPaused();
    if (rp->tryUpdate(m.log_index)) {
      rp->respondedTo();
      if (tryCommit()) broadcastReplicateMessage();
      else if (paused) sendReplicateMessage(m.from);
      // rp may have been invalidated? no: maps are not modified by the above.
      if (leaderTransfering() && m.from == leaderTransferTarget && log.lastIndex() == rp->match)
        sendTimeoutNowMessage(leaderTransferTarget);
    }
  } else {
    if (rp->decreaseTo(m.log_index, m.hint)) {
      enterRetryState(rp);
      sendReplicateMessage(m.from);
    }
  }
}

void Raft::handleLeaderHeartbeatResp(const Message& m, Remote* rp) {  // raft.go:1698-1710
  mustBeLeader();
  rp->setActive();
  rp->waitToRetry();
  if (rp->match < log.lastIndex()) sendReplicateMessage(m.from);
  if (m.hint != 0) handleReadIndexLeaderConfirmation(m);
}

void Raft::handleLeaderTransfer(const Message& m, Remote* rp) {  // raft.go:1712-1734
  mustBeLeader();
  u64 target = m.hint;
  if (target == NoNode) panicf("leader transfer target not set");
  if (leaderTransfering()) return;
  if (nodeID == target) return;
  leaderTransferTarget = target;
  electionTick = 0;
  if (rp->match == log.lastIndex()) sendTimeoutNowMessage(target);
}

void Raft::handleReadIndexLeaderConfirmation(const Message& m) {  // raft.go:1736-1756
  SystemCtx ctx{m.hint, m.hint_high};
  auto ris = readIndex.confirm(ctx, m.from, quorum());
  for (auto& s : ris) {
    if (s.from == NoNode || s.from == nodeID) {
      addReadyToRead(s.index, s.ctx);
    } else {
      Message r;
      r.to = s.from;
      r.type = ReadIndexResp;
      r.log_index = s.index;
      r.hint = m.hint;
      r.hint_high = m.hint_high;
      send(std::move(r));
    }
  }
}

void Raft::handleLeaderSnapshotStatus(const Message& m, Remote* rp) {  // raft.go:1758-1771
  if (rp->state != RemoteSnapshot) return;
  if (m.reject) rp->clearPendingSnapshot();
  rp->becomeWait();
}

void Raft::handleLeaderUnreachable(const Message&, Remote* rp) { enterRetryState(rp); }  // raft.go:1773-1777

void Raft::handleLeaderRateLimit(const Message& m) {  // raft.go:1779-1785
  if (rl.enabled()) rl.setFollowerState(m.from, m.hint);
  // else: dropped (rl disabled)
}

void Raft::sendRateLimitMessage() {  // raft.go:660-683
  if (isLeader()) panicf("leader node called sendRateLimitMessage");
  if (leaderID == NoLeader) return;  // skipped, no leader
  if (!rl.enabled()) return;
  u64 mv = 0;
  if (rl.rateLimited()) {
    // max(inmemSz-notCommitedSz, 0) on uint64: the difference wraps
    mv = rl.get() - entrySliceSize(log.getUncommittedEntries());
  }
  Message m;
  m.type = RateLimit;
  m.to = leaderID;
  m.hint = mv;
  send(m);
}

void Raft::handleFollowerPropose(Message& m) {  // raft.go:1841-1853
  if (leaderID == NoLeader) {
    reportDroppedProposal(m);
    return;
  }
  m.to = leaderID;
  send(m);
}

void Raft::handleFollowerReplicate(const Message& m) {  // raft.go:1859-1863
  electionTick = 0;  // leaderIsAvailable
  setLeaderID(m.from);
  handleReplicateMessage(m);
}

void Raft::handleFollowerHeartbeat(const Message& m) {  // raft.go:1865-1869
  electionTick = 0;
  setLeaderID(m.from);
  handleHeartbeatMessage(m);
}

void Raft::handleFollowerReadIndex(Message& m) {  // raft.go:1871-1879
  if (leaderID == NoLeader) {
    reportDroppedReadIndex(m);
    return;
  }
  m.to = leaderID;
  send(m);
}

void Raft::handleFollowerLeaderTransfer(Message& m) {  // raft.go:1881-1888
  if (leaderID == NoLeader) return;
  m.to = leaderID;
  send(m);
}

void Raft::handleFollowerReadIndexResp(const Message& m) {  // raft.go:1890-1898
  SystemCtx ctx{m.hint, m.hint_high};
  electionTick = 0;
  setLeaderID(m.from);
  addReadyToRead(m.log_index, ctx);
}

void Raft::handleFollowerInstallSnapshot(const Message& m) {  // raft.go:1900-1904
  electionTick = 0;
  setLeaderID(m.from);
  handleInstallSnapshotMessage(m);
}

void Raft::handleFollowerTimeoutNow(const Message&) {  // raft.go:1906-1916
  electionTick = randomizedElectionTimeout;
  isLeaderTransferTarget = true;
  tick();
  if (isLeaderTransferTarget) isLeaderTransferTarget = false;
}

void Raft::handleCandidatePropose(const Message& m) { reportDroppedProposal(m); }  // raft.go:1928-1931

void Raft::handleCandidateReadIndex(const Message& m) {  // raft.go:1933-1941
  reportDroppedReadIndex(m);
  droppedReadIndexes.push_back(SystemCtx{m.hint, m.hint_high});
}

void Raft::handleCandidateReplicate(const Message& m) {  // raft.go:1949-1952
  becomeFollower(term, m.from);
  handleReplicateMessage(m);
}

void Raft::handleCandidateInstallSnapshot(const Message& m) {  // raft.go:1954-1957
  becomeFollower(term, m.from);
  handleInstallSnapshotMessage(m);
}

void Raft::handleCandidateHeartbeat(const Message& m) {  // raft.go:1959-1962
  becomeFollower(term, m.from);
  handleHeartbeatMessage(m);
}

void Raft::handleCandidateRequestVoteResp(const Message& m) {  // raft.go:1964-1981
  if (observers.count(m.from)) return;
  int count = handleVoteResp(m.from, m.reject);
  if (count == quorum()) {
    becomeLeader();
    broadcastReplicateMessage();
  } else if ((int)votes.size() - count == quorum()) {
    becomeFollower(term, NoLeader);
  }
}

void Raft::reportDroppedProposal(const Message& m) {  // raft.go:1987-1997
  droppedEntries.insert(droppedEntries.end(), m.entries.begin(), m.entries.end());
  if (hasEvents) events.proposalDropped++;
}

void Raft::reportDroppedReadIndex(const Message& m) {  // raft.go:1999-2012
  droppedReadIndexes.push_back(SystemCtx{m.hint, m.hint_high});
  if (hasEvents) events.readIndexDropped++;
}

Remote* Raft::lookupRemote(u64 from) {  // lw, raft.go:2014-2028
  auto a = remotes.find(from);
  if (a != remotes.end()) return &a->second;
  auto b = observers.find(from);
  if (b != observers.end()) return &b->second;
  auto c = witnesses.find(from);
  if (c != witnesses.end()) return &c->second;
  return nullptr;
}

// defaultHandle + the handler table of initializeHandlerMap, raft.go:2030-2098
void Raft::dispatch(Message& m) {
  switch (state) {
    case Candidate:
      switch (m.type) {
        case Heartbeat: handleCandidateHeartbeat(m); return;
        case Propose: handleCandidatePropose(m); return;
        case ReadIndex: handleCandidateReadIndex(m); return;
        case Replicate: handleCandidateReplicate(m); return;
        case InstallSnapshot: handleCandidateInstallSnapshot(m); return;
        case RequestVoteResp: handleCandidateRequestVoteResp(m); return;
        case Election: handleNodeElection(m); return;
        case RequestVote: handleNodeRequestVote(m); return;
        case ConfigChangeEvent: handleNodeConfigChange(m); return;
        case LocalTick: handleLocalTick(m); return;
        case SnapshotReceived: handleRestoreRemote(m); return;
        default: return;
      }
    case Follower:
      switch (m.type) {
        case Propose: handleFollowerPropose(m); return;
        case Replicate: handleFollowerReplicate(m); return;
        case Heartbeat: handleFollowerHeartbeat(m); return;
        case ReadIndex: handleFollowerReadIndex(m); return;
        case LeaderTransfer: handleFollowerLeaderTransfer(m); return;
        case ReadIndexResp: handleFollowerReadIndexResp(m); return;
        case InstallSnapshot: handleFollowerInstallSnapshot(m); return;
        case Election: handleNodeElection(m); return;
        case RequestVote: handleNodeRequestVote(m); return;
        case TimeoutNow: handleFollowerTimeoutNow(m); return;
        case ConfigChangeEvent: handleNodeConfigChange(m); return;
        case LocalTick: handleLocalTick(m); return;
        case SnapshotReceived: handleRestoreRemote(m); return;
        default: return;
      }
    case Leader: {
      switch (m.type) {
        case LeaderHeartbeat: handleLeaderHeartbeat(m); return;
        case CheckQuorum: handleLeaderCheckQuorum(m); return;
        case Propose: handleLeaderPropose(m); return;
        case ReadIndex: handleLeaderReadIndex(m); return;
        case ReplicateResp:
        case HeartbeatResp:
        case SnapshotStatus:
        case Unreachable:
        case LeaderTransfer: {
          Remote* rp = lookupRemote(m.from);
          if (rp == nullptr) return;
          if (m.type == ReplicateResp) handleLeaderReplicateResp(m, rp);
          else if (m.type == HeartbeatResp) handleLeaderHeartbeatResp(m, rp);
          else if (m.type == SnapshotStatus) handleLeaderSnapshotStatus(m, rp);
          else if (m.type == Unreachable) handleLeaderUnreachable(m, rp);
          else handleLeaderTransfer(m, rp);
          return;
        }
        case Election: handleNodeElection(m); return;
        case RequestVote: handleNodeRequestVote(m); return;
        case ConfigChangeEvent: handleNodeConfigChange(m); return;
        case LocalTick: handleLocalTick(m); return;
        case SnapshotReceived: handleRestoreRemote(m); return;
        case RateLimit: handleLeaderRateLimit(m); return;
        default: return;
      }
    }
    case Observer:
      switch (m.type) {
        case Heartbeat: handleFollowerHeartbeat(m); return;
        case Replicate: handleFollowerReplicate(m); return;
        case InstallSnapshot: handleFollowerInstallSnapshot(m); return;
        case Propose: handleFollowerPropose(m); return;
        case ReadIndex: handleFollowerReadIndex(m); return;
        case ReadIndexResp: handleFollowerReadIndexResp(m); return;
        case ConfigChangeEvent: handleNodeConfigChange(m); return;
        case LocalTick: handleLocalTick(m); return;
        case SnapshotReceived: handleRestoreRemote(m); return;
        default: return;
      }
    case Witness:
      switch (m.type) {
        case Heartbeat: handleFollowerHeartbeat(m); return;
        case Replicate: handleFollowerReplicate(m); return;
        case InstallSnapshot: handleFollowerInstallSnapshot(m); return;
        case RequestVote: handleNodeRequestVote(m); return;
        case ConfigChangeEvent: handleNodeConfigChange(m); return;
        case LocalTick: handleLocalTick(m); return;
        case SnapshotReceived: handleRestoreRemote(m); return;
        default: return;
      }
    default: return;
  }
}

// ---------------------------------------------------------------- peer.go
Peer* Peer::Launch(const Config& c, ILogDB* logdb,
                   const std::vector<std::pair<u64, std::string>>& addresses,
                   bool initial, bool newNode) {  // peer.go:64-86
  if (c.nodeID == 0) panicf("config.NodeID must not be zero");
  if (initial && newNode && addresses.empty()) panicf("addresses must be specified");
  std::set<std::string> uniq;
  for (auto& a : addresses) uniq.insert(a.second);
  if (uniq.size() != addresses.size()) panicf("duplicated address found");
  Raft* r = new Raft(c, logdb);
  Peer* p = new Peer();
  p->raft = r;
  u64 lastIndex = logdb->GetRange().second;
  if (newNode && !c.isObserver && !c.isWitness) r->becomeFollower(1, NoLeader);
  if (initial && newNode) bootstrap(r, addresses);
  if (lastIndex == 0) p->prevState = PState{};
  else p->prevState = r->raftState();
  return p;
}

void Peer::Tick() {  // peer.go:89-94
  Message m;
  m.type = LocalTick;
  m.reject = false;
  raft->Handle(m);
}

void Peer::QuiescedTick() {  // peer.go:97-102
  Message m;
  m.type = LocalTick;
  m.reject = true;
  raft->Handle(m);
}

void Peer::RequestLeaderTransfer(u64 target) {  // peer.go:106-113
  Message m;
  m.type = LeaderTransfer;
  m.to = raft->nodeID;
  m.from = target;
  m.hint = target;
  raft->Handle(m);
}

void Peer::ProposeEntries(const std::vector<Entry>& ents) {  // peer.go:117-123
  Message m;
  m.type = Propose;
  m.from = raft->nodeID;
  m.entries = ents;
  raft->Handle(m);
}

void Peer::ProposeConfigChange(const std::string& data, u64 key) {  // peer.go:126-135
  Message m;
  m.type = Propose;
  Entry e;
  e.type = ConfigChangeEntry;
  e.cmd = data;
  e.key = key;
  m.entries.push_back(e);
  raft->Handle(m);
}

void Peer::ApplyConfigChange(u64 nodeID, int ccType) {  // peer.go:138-149
  if (nodeID == NoLeader) {
    raft->pendingConfigChange = false;
    return;
  }
  Message m;
  m.type = ConfigChangeEvent;
  m.reject = false;
  m.hint = nodeID;
  m.hint_high = (u64)ccType;
  raft->Handle(m);
}

void Peer::RejectConfigChange() {  // peer.go:152-157
  Message m;
  m.type = ConfigChangeEvent;
  m.reject = true;
  raft->Handle(m);
}

void Peer::RestoreRemotes(const Snapshot& ss) {  // peer.go:160-165
  Message m;
  m.type = SnapshotReceived;
  m.snapshot = ss;
  raft->Handle(m);
}

void Peer::ReportUnreachableNode(u64 nodeID) {  // peer.go:168-173
  Message m;
  m.type = Unreachable;
  m.from = nodeID;
  raft->Handle(m);
}

void Peer::ReportSnapshotStatus(u64 nodeID, bool reject) {  // peer.go:177-183
  Message m;
  m.type = SnapshotStatus;
  m.from = nodeID;
  m.reject = reject;
  raft->Handle(m);
}

void Peer::Handle(const Message& m) {  // peer.go:186-198
  if (isLocalMessageType(m.type)) panicf("local message sent to Step");
  bool rok = raft->remotes.count(m.from) > 0;
  bool ook = raft->observers.count(m.from) > 0;
  bool wok = raft->witnesses.count(m.from) > 0;
  if (rok || ook || wok || !isResponseMessageType(m.type)) raft->Handle(m);
}

Update Peer::GetUpdate(bool moreToApply, u64 lastApplied) {  // peer.go:201-207
  Update ud = getUpdate(moreToApply, lastApplied);
  validateUpdate(ud);
  ud = setFastApply(ud);
  ud.update_commit = getUpdateCommit(ud);
  return ud;
}

Update setFastApply(Update ud) {  // peer.go:209-226
  ud.fast_apply = true;
  if (!isEmptySnapshot(ud.snapshot)) ud.fast_apply = false;
  if (ud.fast_apply) {
    if (!ud.committed_entries.empty() && !ud.entries_to_save.empty()) {
      u64 lastApplyIndex = ud.committed_entries.back().index;
      u64 lastSaveIndex = ud.entries_to_save.back().index;
      u64 firstSaveIndex = ud.entries_to_save[0].index;
      if (lastApplyIndex >= firstSaveIndex && lastApplyIndex <= lastSaveIndex)
        ud.fast_apply = false;
    }
  }
  return ud;
}

void validateUpdate(const Update& ud) {  // peer.go:228-245
  if (ud.state.commit > 0 && !ud.committed_entries.empty()) {
    u64 li = ud.committed_entries.back().index;
    if (li > ud.state.commit) panicf("trying to apply not committed entry");
  }
  if (!ud.committed_entries.empty() && !ud.entries_to_save.empty()) {
    u64 lastApply = ud.committed_entries.back().index;
    u64 lastSave = ud.entries_to_save.back().index;
    if (lastApply > lastSave) panicf("trying to apply not saved entry");
  }
}

bool Peer::HasUpdate(bool moreEntriesToApply) const {  // peer.go:253-280
  Raft* r = raft;
  PState pst = r->raftState();
  if (!isEmptyState(pst) && !isStateEqual(pst, prevState)) return true;
  if (r->log.inmem.hasSnapshot && !isEmptySnapshot(r->log.inmem.snapshot)) return true;
  if (!r->msgs.empty()) return true;
  if (!r->log.entriesToSave().empty()) return true;
  if (moreEntriesToApply && r->log.hasEntriesToApply()) return true;
  if (!r->readyToRead.empty()) return true;
  if (!r->droppedEntries.empty() || !r->droppedReadIndexes.empty()) return true;
  return false;
}

void Peer::Commit(const Update& ud) {  // peer.go:282-293
  raft->msgs.clear();
  raft->droppedEntries.clear();
  raft->droppedReadIndexes.clear();
  if (!isEmptyState(ud.state)) prevState = ud.state;
  if (ud.update_commit.ready_to_read > 0) raft->readyToRead.clear();
  raft->log.commitUpdate(ud.update_commit);
}

void Peer::ReadIndex(SystemCtx ctx) {  // peer.go:297-303
  Message m;
  m.type = orc::ReadIndex;
  m.hint = ctx.low;
  m.hint_high = ctx.high;
  raft->Handle(m);
}

Update Peer::getUpdate(bool moreEntriesToApply, u64 lastApplied) const {  // peer.go:326-358
  Update ud;
  ud.cluster_id = raft->clusterID;
  ud.node_id = raft->nodeID;
  ud.entries_to_save = raft->log.entriesToSave();
  ud.messages = raft->msgs;
  ud.last_applied = lastApplied;
  ud.fast_apply = true;
  if (moreEntriesToApply) ud.committed_entries = raft->log.entriesToApply();
  if (!ud.committed_entries.empty()) {
    u64 li = ud.committed_entries.back().index;
    ud.more_committed_entries = raft->log.hasMoreEntriesToApply(li);
  }
  PState pst = raft->raftState();
  if (!isStateEqual(pst, prevState)) ud.state = pst;
  if (raft->log.inmem.hasSnapshot) ud.snapshot = raft->log.inmem.snapshot;
  if (!raft->readyToRead.empty()) ud.ready_to_reads = raft->readyToRead;
  if (!raft->droppedEntries.empty()) ud.dropped_entries = raft->droppedEntries;
  if (!raft->droppedReadIndexes.empty()) ud.dropped_read_indexes = raft->droppedReadIndexes;
  return ud;
}

void bootstrap(Raft* r, std::vector<std::pair<u64, std::string>> addresses) {  // peer.go:378-408
  std::sort(addresses.begin(), addresses.end(),
            [](const std::pair<u64, std::string>& a, const std::pair<u64, std::string>& b) {
              return a.first < b.first;
            });
  std::vector<Entry> ents(addresses.size());
  for (size_t i = 0; i < addresses.size(); i++) {
    ents[i].type = ConfigChangeEntry;
    ents[i].term = 1;
    ents[i].index = i + 1;
    // Cmd = marshaled ConfigChange{AddNode, NodeID, Initialize, Address}; the raft
    // core never reads it.  Stand-in shared with the engine: 8 bytes, LE of
    // 0xCC00000000000000 | NodeID.
    u64 w = 0xCC00000000000000ULL | addresses[i].first;
    ents[i].cmd.assign(8, '\0');
    for (int b = 0; b < 8; b++) ents[i].cmd[b] = (char)((w >> (8 * b)) & 0xff);
  }
  r->log.append(ents);
  r->log.committed = ents.size();
  for (auto& a : addresses) r->addNode(a.first);
}

UpdateCommit getUpdateCommit(const Update& ud) {  // peer.go:410-427
  UpdateCommit uc;
  uc.ready_to_read = ud.ready_to_reads.size();
  uc.last_applied = ud.last_applied;
  if (!ud.committed_entries.empty()) uc.processed = ud.committed_entries.back().index;
  if (!ud.entries_to_save.empty()) {
    uc.stable_log_to = ud.entries_to_save.back().index;
    uc.stable_log_term = ud.entries_to_save.back().term;
  }
  if (!isEmptySnapshot(ud.snapshot)) {
    uc.stable_snapshot_to = ud.snapshot.index;
    uc.processed = umax(uc.processed, uc.stable_snapshot_to);
  }
  return uc;
}

}  // namespace orc
