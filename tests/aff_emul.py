"""Test infrastructure: the device's affinity-table lookups restated in numpy.

Used only by the CPU tests to pin the exporter's tables (scheduler_amd/affinity.py) against the
oracle before any GPU time: per node, the inter-pod affinity predicate reasons and the normalised
InterPodAffinity score a spec would get from the tables, and the table updates one commit applies.
"""
from __future__ import annotations

import numpy as np

from scheduler_amd import affinity as A

R_POD_AFFINITY, R_EXISTING_ANTI, R_AFFINITY_RULES, R_ANTI_RULES, R_HOST_ERROR = 12, 13, 14, 15, 16


class Tables:
    def __init__(self, snap):
        a = snap.aff
        self.a = a
        self.counters = a.counters.astype(np.int64).copy()
        self.totals = a.totals.astype(np.int64).copy()
        self.h = a.h.astype(np.int64).copy()

    def reasons(self, spec):
        """Reason mask of the inter-pod affinity predicate per node (0 = passes)."""
        a = self.a
        row = a.spec_arr[spec]
        n = a.topo_dom.shape[1]
        out = np.zeros(n, np.int64)
        for c in a.check_arr[row["check_off"]:row["check_off"] + row["check_cnt"]]:
            t = a.table_arr[c["table"]]
            dom = a.topo_dom[t["slot"]]
            cnt = np.where(dom >= 0, self.counters[t["cnt_off"] + np.maximum(dom, 0)], 0)
            undecided = out == 0
            if c["kind"] == A.AFF_EXISTING_ANTI:
                fail = cnt > 0
                bits = (1 << R_POD_AFFINITY) | (1 << R_EXISTING_ANTI)
            elif c["kind"] == A.AFF_ANTI:
                fail = cnt > 0
                bits = (1 << R_POD_AFFINITY) | (1 << R_ANTI_RULES)
            elif c["kind"] == A.AFF_ERROR:  # the reference's predicate returns a plain error
                fail = cnt > 0
                bits = 1 << R_HOST_ERROR
            else:
                match = cnt > 0
                fail = ~match & ((self.totals[c["table"]] > 0) | (row["self_match"] == 0))
                bits = (1 << R_POD_AFFINITY) | (1 << R_AFFINITY_RULES)
            out[undecided & fail] = bits
        return out

    def ipa(self, spec):
        """InterPodAffinity priority per node (interpod_affinity.go:221-238), before the plugin weight."""
        a = self.a
        row = a.spec_arr[spec]
        n = a.topo_dom.shape[1]
        cnt = np.zeros(n, np.int64)
        for h in a.hist_arr[row["hist_off"]:row["hist_off"] + row["hist_cnt"]]:
            dom = a.topo_dom[h["slot"]]
            cnt += np.where(dom >= 0, self.h[h["h_off"] + np.maximum(dom, 0)], 0)
        mx, mn = max(0, int(cnt.max())), min(0, int(cnt.min()))
        if mx - mn <= 0:
            return np.zeros(n, np.int64)
        return np.array([int(10.0 * ((float(c) - mn) / float(mx - mn))) for c in cnt], np.int64)

    def commit(self, spec, node, allocate):
        """Table updates of one placement (Allocate adds to the lister; every commit adds the pod)."""
        a = self.a
        row = a.spec_arr[spec]
        if allocate:
            for t in a.lister_arr[row["lister_off"]:row["lister_off"] + row["lister_cnt"]]:
                tt = a.table_arr[t]
                d = a.topo_dom[tt["slot"], node]
                if d >= 0:
                    self.counters[tt["cnt_off"] + d] += 1
                self.totals[t] += 1
        for e in a.incr_arr[row["incr_off"]:row["incr_off"] + row["incr_cnt"]]:
            d = a.topo_dom[e["slot"], node]
            if d >= 0:
                self.h[e["h_off"] + d] += e["weight"]
