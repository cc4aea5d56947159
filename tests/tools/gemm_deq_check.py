# The register a real dequeue (rn_deq_issue, returning) writes must not be touched by anything but
# rn_deq_noop / rn_deq_take between the issue and the take (loop order: take ... issue ... | back-edge).
import re, sys
bad = 0
for f in sys.argv[1:]:
    lines = open(f).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_ZN14rn_gemm_detail7gemm_pk\S+:", l)]
    starts.append(len(lines))
    for a, b in zip(starts, starts[1:]):
        body = lines[a:b]
        iss = [i for i, l in enumerate(body) if "rn_deq_issue" in l]
        tak = [i for i, l in enumerate(body) if "rn_deq_take" in l]
        if not iss:
            continue
        reg = re.search(r"buffer_atomic_add (v\d+),", body[iss[0]]).group(1)
        treg = re.search(r"rn_deq_take (v\d+)", body[tak[0]]).group(1)
        # loop header = last label before the take that is a loop header
        hdr = max(i for i in range(tak[0]) if re.match(r"^\.LBB\S+:.*Loop Header|^\.LBB\S+:\s+; %bb", body[i]) or "Loop Header" in body[i])
        end = max(i for i, l in enumerate(body) if "s_cbranch" in l and l.split()[-1].rstrip(":") in body[hdr])
        window = list(range(iss[0] + 1, end + 1)) + list(range(hdr, tak[0]))
        touch = [(i, body[i].strip()) for i in window if re.search(rf"\b{reg}\b", body[i])
                 and "rn_deq_noop" not in body[i] and "rn_deq_take" not in body[i]]
        ok = reg == treg and not touch
        bad += not ok
        print(f"{f.split('/')[-1]} {lines[a][28:70]} reg={reg} take={treg} touches={touch[:3]} {'OK' if ok else 'BAD'}")
sys.exit(1 if bad else 0)
