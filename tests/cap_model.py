"""A CPU model of csrc/capmask.h's cap_walk_kernel, lane for lane.

The wave's logic (chunks of 64 reads, the bulk path, groups in lane order,
the LDS ring of read ends and its pointer) restated over Python lists, so
the device walk's control flow can be checked against the host closed form
(mc_depth_cap_mask) on any pile without a GPU (tests/test_depth_cap.py).
`ring` is the ring size (the kernel's kCapRing; small rings exercise the
wrap-around and the gap paths).
"""


def cap_walk(pos, span, inq, max_depth, max_span, ring=32768):
    n = len(pos)
    mask = ring - 1
    E = [0] * ring
    st = {"total": 0, "removed": 0, "ptr": 0, "have_ptr": False}

    def advance(s):
        if not st["have_ptr"]:
            st["ptr"], st["have_ptr"] = s, True
            return
        if s <= st["ptr"]:
            return
        m = s - st["ptr"]
        acc = 0
        if m >= ring:
            for k in range(ring):
                acc += E[k]
                E[k] = 0
        else:
            for x in range(m):
                k = (st["ptr"] + x) & mask
                acc += E[k]
                E[k] = 0
        st["removed"] += acc
        st["ptr"] = s

    keep = [0] * n
    out_span = list(span)
    C = b = 0
    last_pos, have_last = 0, False
    dropped = 0
    for c0 in range(0, n, 64):
        lanes = range(64)
        valid = [c0 + l < n for l in lanes]
        p = [pos[c0 + l] if valid[l] else 0 for l in lanes]
        sp = [span[c0 + l] if valid[l] else 0 for l in lanes]
        q = [valid[l] and bool(inq[c0 + l]) for l in lanes]
        kept = [False] * 64
        if any(q):
            gstart = [False] * 64
            prev = None
            for l in lanes:
                if not q[l]:
                    continue
                pp = prev if prev is not None else (last_pos if have_last else None)
                gstart[l] = pp is None or p[l] != pp
                prev = p[l]
            gl = [l for l in lanes if gstart[l]]
            live = st["total"] - st["removed"]
            if gl:
                s_first, s_last = p[gl[0]], p[gl[-1]]
                base = st["ptr"] if st["have_ptr"] else s_first
                fits = s_last - base + max_span + 64 < ring
            else:
                fits = True
            if live + 64 <= max_depth and fits:
                if gl and not st["have_ptr"]:
                    advance(s_first)
                u = [q[l] and (gstart[l] or sp[l] > 0) for l in lanes]
                for l in lanes:
                    if u[l]:
                        E[(p[l] + sp[l]) & mask] += 1
                st["total"] += sum(u)
                kept = list(q)
                if gl:
                    advance(s_last)
                    b = sum(1 for l in lanes if u[l] and l >= gl[-1])
                    C = st["total"] - st["removed"] - b
                else:
                    b += sum(u)
            else:
                parts = []
                cont = [l for l in lanes if q[l] and (not gl or l < gl[0])]
                parts.append((None, cont))
                for k, g in enumerate(gl):
                    end = gl[k + 1] if k + 1 < len(gl) else 64
                    parts.append((g, [l for l in range(g, end) if q[l]]))
                for first, part in parts:
                    if first is not None:
                        advance(p[first])
                        C = st["total"] - st["removed"]
                        b = 0
                    if not part:
                        continue
                    u = {l: (l == first or sp[l] > 0) for l in part}
                    ks = {}
                    for l in part:
                        bb = b + sum(1 for m in part if m < l and u[m])
                        ks[l] = l == first or 1 + C + bb <= max_depth
                    for l in part:
                        if ks[l] and u[l]:
                            E[(p[l] + sp[l]) & mask] += 1
                    t = sum(1 for l in part if ks[l] and u[l])
                    st["total"] += t
                    b += t
                    dropped += sum(1 for l in part if not ks[l])
                    for l in part:
                        kept[l] = ks[l]
            last_pos = p[max(l for l in lanes if q[l])]
            have_last = True
        for l in lanes:
            if valid[l]:
                keep[c0 + l] = 1 if kept[l] else 0
                if not kept[l] and sp[l] != 0:
                    out_span[c0 + l] = 0
    return keep, out_span, dropped
