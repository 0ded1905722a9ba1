"""Learn reliability (member) restated in Python — TEST INFRASTRUCTURE (oracle/: only tests use it, as the checker).

The engine's mpx_read_learns (engine.cpp learn_plan + kernels.hip k_learns) in plain
loops over a trace and its MPXR result: the promise quorums and chosen batches the
MPXR records stand for what the device computes (F_QUORUM, k_votes).  Checked against
the reference's own bookkeeping (tests/golden/*.mpxl, oracle/ref_member_driver.cpp) on
CPU, so the algorithm is pinned before the GPU runs it.  member/paxos.cpp lines cited.
"""
import struct

import mpxr

NONE = (1 << 64) - 1


def _streams(trace):
    ver, n = struct.unpack_from("<II", trace, 4)
    ne = struct.unpack_from("<I", trace, 24)[0]
    esz = 24 if ver == 1 else 32
    epochs = []
    for i in range(ne):
        v, a, p = struct.unpack_from("<IxxxxQQ", trace, 40 + esz * i)
        lm = struct.unpack_from("<Q", trace, 40 + esz * i + 24)[0] if esz == 32 else p
        epochs.append((v, a, p, lm))
    pos = 40 + esz * ne
    streams = []
    for _ in range(n):
        cnt, nb = struct.unpack_from("<QQ", trace, pos)
        offs = struct.unpack_from("<%dQ" % (cnt + 1), trace, pos + 16)
        body = pos + 16 + 8 * (cnt + 1)
        streams.append([bytes(trace[body + offs[k]: body + offs[k + 1]]) for k in range(cnt)])
        pos = (body + nb + 7) & ~7
    return epochs, streams


def learns(trace, result):
    epochs, streams = _streams(trace)
    res = mpxr.parse(result)
    out = []
    for n, msgs in enumerate(streams):
        quorum_at = {q[0] for q in res["nodes"][n]["quorums"]}
        chosen_at = dict(res["nodes"][n]["chosen_batches"])
        recs = []                       # [id, created, kind, src, facc, end, events]
        live = []
        st = {"ei": 0, "prop": bool((epochs[0][2] >> n) & 1), "prep": False, "lid": 0,
              "amask": epochs[0][1], "learned_any": False}

        def create(at, kind, src, facc):
            st["lid"] += 1
            live.append(len(recs))
            recs.append([st["lid"], at, kind, src, facc, NONE, []])

        def drop_all(at):
            for x in live:
                recs[x][5] = at
            live.clear()

        def acc_changed(at, who, add):          # AcceptorsChanged (:1504-1549)
            for x in live:
                if recs[x][4]:
                    recs[x][6].append(("acc", at, who, add, st["amask"]))
            st["prep"] = True

        def learners_changed(at):               # LearnersChanged (:1472-1502)
            drop_all(at)
            if not st["prep"]:
                create(at, 2, 0, True)

        K = 0
        idle = False
        for k, m in enumerate(msgs):
            t = struct.unpack_from("<I", m)[0]
            if t != 18:
                K = k
                if idle:                        # after the whole marker run (see below)
                    st["prep"], idle = False, False
            if t == 1 and k in quorum_at:
                st["prep"] = False
                if st["learned_any"]:
                    create(k, 1, 0, True)
            elif t == 4 and k in chosen_at:
                create(k, 0, chosen_at[k], False)
            elif t == 6:
                if not st["prop"]:
                    continue
                learner, lid = struct.unpack_from("<IQ", m, 4)
                lc = bin(epochs[st["ei"]][3]).count("1")
                for x in live:
                    if recs[x][0] == lid:
                        recs[x][6].append(("reply", k, learner, lc, st["amask"]))
            elif t == 16:
                if st["prop"]:
                    st["prep"] = True
            elif t == 5:
                if struct.unpack_from("<I", m, 16)[0]:
                    st["learned_any"] = True
            elif t == 18:
                ej = struct.unpack_from("<I", m, 4)[0]
                o, x = epochs[st["ei"]], epochs[ej]
                was, now = bool((o[2] >> n) & 1), bool((x[2] >> n) & 1)
                gl, ll = x[3] & ~o[3], o[3] & ~x[3]
                ga, la = x[1] & ~o[1], o[1] & ~x[1]
                assert not ((gl or ga or (now and not was)) and (ll or la or (was and not now)))
                for b in range(64):
                    if (gl >> b) & 1 and st["prop"]:
                        learners_changed(K)
                if now and not was:
                    st.update(prop=True, lid=0, prep=False)
                    live.clear()
                for b in range(64):
                    if (ga >> b) & 1:
                        st["amask"] |= 1 << b
                        if st["prop"]:
                            acc_changed(K, b, True)
                for b in range(64):
                    if (la >> b) & 1:
                        st["amask"] &= ~(1 << b)
                        if st["prop"]:
                            acc_changed(K, b, False)
                if was and not now:
                    drop_all(K)
                    st["prop"] = False
                for b in range(64):
                    if (ll >> b) & 1 and st["prop"]:
                        learners_changed(K)
                st["amask"] = x[1]
                # the engine model's idle proposer: the driver idles it at each marker, once
                # every change of the LEARN has run, so it takes effect after the marker run
                if now and (not was or o[1] != x[1]):
                    idle = True
                st["ei"] = ej
        rows = []
        for lid, created, kind, src, facc, end, evs in recs:
            learned = acc = 0
            applied = retired = NONE
            for ev in evs:
                am = ev[4]
                q = bin(am).count("1") // 2 + 1
                if ev[0] == "reply":
                    _, at, who, lc, _ = ev
                    learned |= 1 << who                              # :1353
                    if facc and (am >> who) & 1:                     # :1355-1370
                        acc |= 1 << who
                        if bin(acc).count("1") >= q:
                            applied, facc = at, False
                    if bin(learned).count("1") == lc:                # :1373-1380
                        retired = at
                        break
                elif facc:
                    _, at, who, add, _ = ev
                    if add:
                        if (learned >> who) & 1:
                            acc |= 1 << who
                    else:
                        acc &= ~(1 << who)
                    if bin(acc).count("1") >= q:                     # :1521-1528
                        applied, facc = at, False
            rows.append((lid, created, kind, src, applied, retired, end if retired == NONE else NONE, learned))
        out.append(rows)
    b = bytearray(b"MPXL") + struct.pack("<II", 1, len(out))
    for rows in out:
        b += struct.pack("<Q", len(rows))
        for r in rows:
            b += struct.pack("<8Q", *r)
    return bytes(b)
