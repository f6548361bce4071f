// dm_server.cpp — round-oriented GetCapacity dispatch over the device-resident
// store (include/doorman_hip.h, "round-oriented GetCapacity dispatch").
//
// The reference serves each ResourceRequest with its own Resource.Decide
// (server.go:798-817 -> resource.go:100-113): Clean, then Learn or the
// resource's Algorithm against the live store, then Assign.  Here a round's
// requests are queued, and dm_server_tick decides them together on the GPU:
//
//   1. Clean (store.go:169-181): leases whose expiry passed are released and
//      their clients forgotten; ReleaseCapacity (server.go:668-714) likewise.
//   2. New clients take a free row (no lease: store.HasClient is false for them).
//   3. dm_decide runs Resource.Decide for every request of the round in queue
//      order -- the request's own has (Learn), wants and subclients for its
//      client, the stored rows for everyone else (algorithm.go:115,148,157,
//      223-225,263-269) -- and each decision's Assign is seen by the requests
//      after it on the same resource, as res.mu serialises the reference's
//      GetCapacity calls (resource.go:103-104).  The round's final leases are
//      then written to the store (dm_store_upsert, store.go:153-167: sums +=
//      new - old, expiry = now + length).  A round is exactly the reference
//      serving its requests one after another in queue order.
//
// Clients that did not ask this round keep their leases (and count in the
// sums) until they expire.  The host keeps the client -> row maps, the rows'
// lease mirror (has, expiry) and a min-heap of expiries, so Clean costs
// O(expired log N), not a scan.  A resource that runs out of free rows grows:
// the table is re-laid out with the resource's segment doubled, the running
// sums carried over exactly (dm_read_resources -> dm_store_load aggregates).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/doorman_hip.h"

namespace {

struct Req {
  int64_t res;
  std::string client;
  double has, wants;
  int64_t sub;
};

struct Out {
  double capacity = 0.0, safe = NAN;
  int64_t expiry_s = 0, refresh_s = 0;
};

}  // namespace

struct dm_server {
  dm_ctx* ctx = nullptr;
  std::string err;
  int64_t R = 0;
  std::unordered_map<std::string, int64_t> res_index;
  // configuration (host copy, dm_resource_cfg columns)
  std::vector<int32_t> kind;
  std::vector<double> capacity, safe_capacity;
  std::vector<int64_t> lease_s, refresh_s, learning_end, parent_expiry;
  // table layout and host mirror
  std::vector<int64_t> seg_off;                                   // R+1
  std::vector<std::unordered_map<std::string, int64_t>> clients;  // per resource: client -> row
  std::vector<std::vector<int64_t>> free_rows;                    // per resource
  std::vector<double> has;                                        // per row: the assigned lease
  std::vector<int64_t> expiry;                                    // per row; DM_RELEASED = free
  std::vector<std::string> row_client;
  // Clean: (expiry, row) min-heap; stale entries are skipped
  std::priority_queue<std::pair<int64_t, int64_t>, std::vector<std::pair<int64_t, int64_t>>, std::greater<>> heap;
  // the current round
  std::vector<Req> pending;
  std::vector<std::pair<int64_t, std::string>> releases;
  std::vector<Out> results;
  std::string broken;  // set when a re-layout failed half way: every later tick refuses

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int ctx_fail(int code) {
    err = dm_last_error(ctx);
    return code;
  }
  int64_t N() const { return seg_off.empty() ? 0 : seg_off.back(); }
  dm_resource_cfg cfg() const {
    return dm_resource_cfg{kind.data(),         capacity.data(),      lease_s.data(),       refresh_s.data(),
                           learning_end.data(), parent_expiry.data(), safe_capacity.data()};
  }
};

namespace {

// (Re)load the table with segment sizes `sizes`, carrying every client's row
// (wants, has, subclients, expiry) and the running sums of the old layout.
int relayout(dm_server* s, const std::vector<int64_t>& sizes) {
  const int64_t R = s->R, oldN = s->N();
  std::vector<double> o_has(oldN), o_wants(oldN);
  std::vector<int64_t> o_sub(oldN), o_exp(oldN);
  std::vector<int64_t> cnt(R, 0);
  std::vector<double> sh(R, 0.0), sw(R, 0.0);
  if (oldN > 0) {
    int rc = dm_read_store(s->ctx, 0, oldN, o_has.data(), o_wants.data(), o_sub.data(), o_exp.data());
    if (rc) return s->ctx_fail(rc);
    rc = dm_read_resources(s->ctx, 0, R, cnt.data(), sh.data(), sw.data(), nullptr);
    if (rc) return s->ctx_fail(rc);
  }
  std::vector<int64_t> off(R + 1, 0);
  for (int64_t r = 0; r < R; ++r) off[r + 1] = off[r] + sizes[r];
  const int64_t N = off[R];
  std::vector<double> n_has(N, 0.0), n_wants(N, 0.0);
  std::vector<int64_t> n_sub(N, 0), n_exp(N, DM_RELEASED);
  std::vector<std::string> n_client(N);
  std::vector<double> m_has(N, 0.0);
  for (int64_t r = 0; r < R; ++r) {
    int64_t next = off[r];
    auto& cl = s->clients[r];
    for (auto& kv : cl) {
      const int64_t o = kv.second, row = next++;
      n_has[row] = o_has[o];
      n_wants[row] = o_wants[o];
      n_sub[row] = o_sub[o];
      n_exp[row] = o_exp[o];
      n_client[row] = kv.first;
      m_has[row] = s->has[o];
      kv.second = row;
    }
    s->free_rows[r].clear();
    for (int64_t row = off[r + 1] - 1; row >= next; --row) s->free_rows[r].push_back(row);
  }
  dm_snapshot snap{R, N, off.data(), n_wants.data(), n_has.data(), n_sub.data(), n_exp.data(),
                   cnt.data(), sh.data(), sw.data()};
  int rc = dm_store_load(s->ctx, &snap);
  if (rc) return s->ctx_fail(rc);
  const dm_resource_cfg cfg = s->cfg();
  rc = dm_config_load(s->ctx, R, &cfg);
  if (rc) return s->ctx_fail(rc);
  s->seg_off = off;
  s->has = m_has;
  s->expiry = n_exp;
  s->row_client = n_client;
  s->heap = {};
  for (int64_t row = 0; row < N; ++row)
    if (n_exp[row] != DM_RELEASED) s->heap.push({n_exp[row], row});
  return DM_OK;
}

int release_rows(dm_server* s, std::vector<int64_t>& rows) {
  if (rows.empty()) return DM_OK;
  std::sort(rows.begin(), rows.end());
  rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
  const int rc = dm_store_release(s->ctx, (int64_t)rows.size(), rows.data());
  if (rc) return s->ctx_fail(rc);
  for (int64_t row : rows) {
    const int64_t r = std::upper_bound(s->seg_off.begin(), s->seg_off.end(), row) - s->seg_off.begin() - 1;
    s->clients[r].erase(s->row_client[row]);
    s->row_client[row].clear();
    s->has[row] = 0.0;
    s->expiry[row] = DM_RELEASED;
    s->free_rows[r].push_back(row);
  }
  return DM_OK;
}

}  // namespace

extern "C" {

int dm_server_create(int device, int64_t n_resources, const char* const* ids, const dm_resource_cfg* cfg,
                     int64_t slots, dm_server** out) {
  if (!out || n_resources < 0 || (n_resources > 0 && (!ids || !cfg)) || slots < 1) return DM_E_INVAL;
  *out = nullptr;
  dm_server* s = new dm_server();
  int rc = dm_create(device, &s->ctx);
  if (rc) {
    delete s;
    return rc;
  }
  const int64_t R = n_resources;
  s->R = R;
  for (int64_t r = 0; r < R; ++r) {
    if (!ids[r] || !s->res_index.emplace(ids[r], r).second) {
      dm_server_destroy(s);
      return DM_E_INVAL;  // missing or duplicate resource id
    }
  }
  s->kind.assign(cfg->kind, cfg->kind + R);
  s->capacity.assign(cfg->capacity, cfg->capacity + R);
  s->safe_capacity.assign(cfg->safe_capacity, cfg->safe_capacity + R);
  s->lease_s.assign(cfg->lease_length_s, cfg->lease_length_s + R);
  s->refresh_s.assign(cfg->refresh_interval_s, cfg->refresh_interval_s + R);
  s->learning_end.assign(cfg->learning_end_ns, cfg->learning_end_ns + R);
  s->parent_expiry.assign(cfg->parent_expiry_ns, cfg->parent_expiry_ns + R);
  s->clients.assign(R, {});
  s->free_rows.assign(R, {});
  rc = relayout(s, std::vector<int64_t>(R, slots));
  if (rc) {
    dm_server_destroy(s);
    return rc;
  }
  *out = s;
  return DM_OK;
}

void dm_server_destroy(dm_server* s) {
  if (!s) return;
  if (s->ctx) dm_destroy(s->ctx);
  delete s;
}

const char* dm_server_last_error(dm_server* s) { return s ? s->err.c_str() : "null server"; }

dm_ctx* dm_server_ctx(dm_server* s) { return s ? s->ctx : nullptr; }

int dm_server_get_capacity(dm_server* s, const char* client, const char* resource, double has, double wants,
                           int64_t subclients, int64_t* ticket) {
  if (!s || !client || !resource || !ticket) return DM_E_INVAL;
  auto it = s->res_index.find(resource);
  if (it == s->res_index.end()) return s->fail(DM_E_RANGE, std::string("unknown resource ") + resource);
  if (subclients < 1 || subclients > 2147483646LL)  // the store's column holds [0, 2^31 - 2] (dm_device.h)
    return s->fail(DM_E_ARGUMENT, "subclients must be in [1, 2^31 - 1) (server.go:863-866)");
  *ticket = (int64_t)s->pending.size();
  s->pending.push_back(Req{it->second, client, has, wants, subclients});
  return DM_OK;
}

int dm_server_release_capacity(dm_server* s, const char* client, const char* resource) {
  if (!s || !client || !resource) return DM_E_INVAL;
  auto it = s->res_index.find(resource);
  if (it == s->res_index.end()) return DM_OK;  // the reference ignores unknown resources (server.go:706-710)
  s->releases.emplace_back(it->second, client);
  return DM_OK;
}

int dm_server_tick(dm_server* s, int64_t now) {
  if (!s) return DM_E_INVAL;
  s->results.clear();  // tickets of a round that fails return an error, never stale leases
  std::vector<Req> reqs;
  reqs.swap(s->pending);
  std::vector<std::pair<int64_t, std::string>> rels;
  rels.swap(s->releases);
  if (!s->broken.empty()) return s->fail(DM_E_STATE, "server unusable after a failed re-layout: " + s->broken);
  int rc;
  // 1. Clean (strict After: now > expiry) and ReleaseCapacity
  std::vector<std::pair<int64_t, int64_t>> popped;
  std::vector<int64_t> drop;
  while (!s->heap.empty() && s->heap.top().first < now) {
    const auto e = s->heap.top();
    s->heap.pop();
    popped.push_back(e);
    if (s->expiry[e.second] == e.first && !s->row_client[e.second].empty()) drop.push_back(e.second);
  }
  for (auto& rel : rels) {
    auto c = s->clients[rel.first].find(rel.second);
    if (c != s->clients[rel.first].end()) drop.push_back(c->second);
  }
  if ((rc = release_rows(s, drop))) {  // the store is untouched: put Clean's heap entries back
    for (const auto& e : popped) s->heap.push(e);
    return rc;
  }
  // rows for the requests: grow resources that lack free rows first
  {
    std::vector<int64_t> need(s->R, 0);
    std::unordered_map<std::string, int> seen;
    for (const Req& q : reqs)
      if (!s->clients[q.res].count(q.client) && seen.emplace(std::to_string(q.res) + '/' + q.client, 1).second)
        ++need[q.res];
    bool grow = false;
    std::vector<int64_t> sizes(s->R);
    for (int64_t r = 0; r < s->R; ++r) {
      const int64_t size = s->seg_off[r + 1] - s->seg_off[r];
      sizes[r] = size;
      if (need[r] > (int64_t)s->free_rows[r].size()) {
        grow = true;
        const int64_t used = size - (int64_t)s->free_rows[r].size();
        while (sizes[r] < used + need[r]) sizes[r] = std::max<int64_t>(2 * sizes[r], 1);
      }
    }
    if (grow && (rc = relayout(s, sizes))) {
      s->broken = s->err;  // host mirror and device table may disagree now
      return rc;
    }
  }
  // 2. every request in queue order; a new client takes a free row, which holds no
  //    lease (store.HasClient false for its first decision)
  const int64_t nq = (int64_t)reqs.size();
  std::vector<int64_t> q_row((size_t)nq), q_sub((size_t)nq);
  std::vector<double> q_has((size_t)nq), q_wants((size_t)nq);
  std::unordered_map<int64_t, size_t> row_last;  // row -> the last request on it
  struct Fresh {
    int64_t res, row;
    std::string client;
  };
  std::vector<Fresh> fresh;
  for (size_t k = 0; k < reqs.size(); ++k) {
    const Req& q = reqs[k];
    auto& cl = s->clients[q.res];
    auto c = cl.find(q.client);
    int64_t row;
    if (c == cl.end()) {
      row = s->free_rows[q.res].back();
      s->free_rows[q.res].pop_back();
      cl.emplace(q.client, row);
      s->row_client[row] = q.client;
      fresh.push_back(Fresh{q.res, row, q.client});
    } else {
      row = c->second;
    }
    q_row[k] = row;
    q_has[k] = q.has;
    q_wants[k] = q.wants;
    q_sub[k] = q.sub;
    row_last[row] = k;
  }
  auto rollback = [&](int code) {  // new clients never got a lease: forget them
    for (const Fresh& f : fresh) {
      s->clients[f.res].erase(f.client);
      s->row_client[f.row].clear();
      s->free_rows[f.res].push_back(f.row);
    }
    return s->ctx_fail(code);
  };
  if (nq == 0) return DM_OK;
  // 3. Resource.Decide for every request in queue order, each seeing the Assigns of
  //    the requests before it on its resource (res.mu serialises them,
  //    resource.go:103-104); then the round's final leases go into the store
  //    (store.go:153-167), one Assign per row with its last request's values
  std::vector<double> gets((size_t)nq);
  std::vector<int64_t> exp((size_t)nq);
  if ((rc = dm_decide(s->ctx, now, nq, q_row.data(), q_has.data(), q_wants.data(), q_sub.data(), gets.data(),
                      exp.data())))
    return rollback(rc);
  std::vector<int64_t> rows, u_sub, u_exp;
  std::vector<double> u_gets, u_wants;
  for (int64_t k = 0; k < nq; ++k) {
    if (row_last[q_row[k]] != (size_t)k) continue;
    rows.push_back(q_row[k]);
    u_gets.push_back(gets[k]);
    u_wants.push_back(q_wants[k]);
    u_sub.push_back(q_sub[k]);
    u_exp.push_back(exp[k]);
  }
  const int64_t n = (int64_t)rows.size();
  if ((rc = dm_store_upsert(s->ctx, n, rows.data(), u_gets.data(), u_wants.data(), u_sub.data(), u_exp.data())))
    return rollback(rc);
  for (int64_t j = 0; j < n; ++j) {
    s->has[rows[j]] = u_gets[j];
    s->expiry[rows[j]] = u_exp[j];
    s->heap.push({u_exp[j], rows[j]});
  }
  // SetSafeCapacity (resource.go:81-96) after the round's Assigns
  int64_t rlo = s->R, rhi = -1;
  for (const Req& q : reqs) {
    rlo = std::min(rlo, q.res);
    rhi = std::max(rhi, q.res);
  }
  std::vector<int64_t> count((size_t)(rhi - rlo + 1));
  if ((rc = dm_read_resources(s->ctx, rlo, rhi - rlo + 1, count.data(), nullptr, nullptr, nullptr)))
    return s->ctx_fail(rc);
  s->results.assign(reqs.size(), Out{});
  for (size_t k = 0; k < reqs.size(); ++k) {
    const int64_t r = reqs[k].res;
    Out& o = s->results[k];
    o.capacity = gets[k];
    // Lease.Expiry.Unix() (server.go:789): seconds, rounded toward -inf
    o.expiry_s = exp[k] >= 0 ? exp[k] / 1000000000LL : -((-exp[k] + 999999999LL) / 1000000000LL);
    o.refresh_s = s->refresh_s[r];  // int64(RefreshInterval.Seconds())
    const double safe = s->safe_capacity[r];
    o.safe = std::isnan(safe) ? s->capacity[r] / (double)count[(size_t)(r - rlo)] : safe;
  }
  return DM_OK;
}

int dm_server_lease(dm_server* s, int64_t ticket, double* capacity, int64_t* expiry_time_s, int64_t* refresh_s,
                    double* safe_capacity) {
  if (!s) return DM_E_INVAL;
  if (ticket < 0 || ticket >= (int64_t)s->results.size())
    return s->fail(DM_E_RANGE, "no such ticket (the last round failed, or had fewer requests)");
  const Out& o = s->results[(size_t)ticket];
  if (capacity) *capacity = o.capacity;
  if (expiry_time_s) *expiry_time_s = o.expiry_s;
  if (refresh_s) *refresh_s = o.refresh_s;
  if (safe_capacity) *safe_capacity = o.safe;
  return DM_OK;
}

int dm_server_resource(dm_server* s, const char* resource, int64_t* clients, int64_t* count, double* sum_has,
                       double* sum_wants) {
  if (!s || !resource) return DM_E_INVAL;
  auto it = s->res_index.find(resource);
  if (it == s->res_index.end()) return s->fail(DM_E_RANGE, std::string("unknown resource ") + resource);
  if (clients) *clients = (int64_t)s->clients[it->second].size();
  const int rc = dm_read_resources(s->ctx, it->second, 1, count, sum_has, sum_wants, nullptr);
  return rc ? s->ctx_fail(rc) : DM_OK;
}

}  // extern "C"
