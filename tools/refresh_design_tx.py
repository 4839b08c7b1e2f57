#!/usr/bin/env python3
"""Rewrite the TX / RX / drop-in latency figures in DESIGN.md from the committed profiles
(profiles/r01_tx_latency.jsonl, r01_txq_sweep.jsonl, r01_rxq_bench.jsonl), so the prose and the
results table quote the same run. Documentation helper; run from the repository root."""
import json, re
lat=[json.loads(l) for l in open('profiles/r01_tx_latency.jsonl')]
pin={d['n']:d for d in lat if d['path']=='tx_host_pinned'}
dro={d['len']:d for d in lat if d['path']=='dropin_ether_fcs'}
sw=[json.loads(l) for l in open('profiles/r01_txq_sweep.jsonl')]
rx=[json.loads(l) for l in open('profiles/r01_rxq_bench.jsonl')]
def g(mode,sink,p,pay=1500,lin=0):
    for x in sw:
        if x['mode']==mode and x['sink']==sink and x['producers']==p and x['payload']==pay and x['flush_usec']==lin: return x
    raise KeyError((mode,sink,p,pay,lin))
def r(t,pl,b):
    for x in rx:
        if x['trailer']==t and x['payload']==pl and x['max_batch']==b: return x
    raise KeyError
p='DESIGN.md'; s=open(p).read()
def sub(pattern, repl):
    global s
    n=len(re.findall(pattern, s, flags=re.S))
    assert n==1, (pattern, n)
    s=re.sub(pattern, repl, s, flags=re.S)
sub(r'Round trips \(`profiles/r01_tx_latency.jsonl`\): 128 frames [0-9.]+ µs, 1024 frames [0-9.]+ µs\.',
    f"Round trips (`profiles/r01_tx_latency.jsonl`): 128 frames {pin[128]['us_per_call']:.1f} µs, 1024 frames {pin[1024]['us_per_call']:.1f} µs.")
sub(r'the last one stores the completion word\. 16 frames: [0-9.]+ µs \(was 14\.9',
    f"the last one stores the completion word. 16 frames: {pin[16]['us_per_call']:.1f} µs (was 14.9")
sub(r'not, goes through the drop-in.s single-frame kernel below: [0-9.]+ µs \(was 13\.5\)\. The TX\n  queue.s lone sync producer now sends [0-9]+ k frames/s',
    f"not, goes through the drop-in's single-frame kernel below: {pin[1]['us_per_call']:.1f} µs (was 13.5). The TX\n  queue's lone sync producer now sends {g('txq','null',1)['Mframes_s']*1000:.0f} k frames/s")
sub(r'as well\. Per call: [0-9.]+ µs median, [0-9.]+ µs p99 for 1514 B; [0-9.]+ µs for 64 B',
    f"as well. Per call: {dro[1514]['p50_us']:.1f} µs median, {dro[1514]['p99_us']:.1f} µs p99 for 1514 B; {dro[64]['p50_us']:.1f} µs for 64 B")
sub(r'[0-9.]+ µs for 4000 B; ([0-9.]+–[0-9.]+ µs median over [a-z]+ boxes\))',
    f"{dro[4000]['p50_us']:.1f} µs for 4000 B; \\1")
i=s.index('| TX queue, 1 sync producer, 1500-B payloads |'); j=s.index('\n',i)
s=s[:i]+f"| TX queue, 1 sync producer, 1500-B payloads | {g('txq','null',1)['Mframes_s']*1000:.0f} k frames/s ({1e3/g('txq','null',1)['Mframes_s']/1000:.1f} µs per frame; was 65 k) | per-frame drop-in `ether_fcs`: {dro[1514]['p50_us']:.1f} µs median per 1514-B call (`profiles/r01_tx_latency.jsonl`) |"+s[j:]
s16=g('txq','null',16); s16s=g('txq','socketpair',16)
i=s.index('| TX queue, 16 sync producers |'); j=s.index('\n',i)
s=s[:i]+f"| TX queue, 16 sync producers | {s16['Mframes_s']*1000:.0f} k frames/s, {s16['Gbit_s']:.2f} Gbit/s (was 464 k); {s16s['Mframes_s']*1000:.0f} k frames/s through a socketpair | batches average {s16['mean_batch']:.1f} frames: each caller waits for its own frame's GPU round trip (~11 µs), so a sync batch holds at most one frame per caller (`profiles/r01_txq_sweep.jsonl`) |"+s[j:]
a1=g('async','null',1); a4=g('async','null',4); a8=g('async','null',8); a16=g('async','null',16); ar=g('async','null',8,-1)
i=s.index('| TX queue, async producers (fire-and-forget), null sink |'); j=s.index('\n',i)
s=s[:i]+f"| TX queue, async producers (fire-and-forget), null sink | **{a1['Mframes_s']:.1f} M frames/s (1 producer), {a4['Mframes_s']:.1f} M/s (4), {a8['Mframes_s']:.1f} M/s = {a8['Gbit_s']:.0f} Gbit/s (8), {a16['Mframes_s']:.1f} M/s (16)**; random payloads, 8 producers: {ar['Mframes_s']:.1f} M/s | sharded reservation + in-place batches up to 64 MiB; was 3.8 M/s (4) and 4.4 M/s (8) with one reservation word. Rates move ±15 % between runs with how large the batches grow |"+s[j:]
i=s.index('| RX queue with GPU FCS check'); j=s.index('\n',i)
s=s[:i]+f"| RX queue with GPU FCS check (`fcs_rxq_receive`, trailer on), AF_UNIX socketpair | **{r(1,1500,64)['Mframes_s']:.2f} M frames/s at batch 64, {r(1,1500,512)['Mframes_s']:.2f} M/s = {r(1,1500,512)['Gbit_s']:.0f} Gbit/s at 512** (1500-B payloads); {r(1,64,512)['Mframes_s']:.2f} M/s with 64-B payloads | check overlapped with the next `recvmmsg`; the socket alone: {r(0,1500,64)['Mframes_s']:.2f} / {r(0,64,512)['Mframes_s']:.2f} M/s (`profiles/r01_rxq_bench.jsonl`) |"+s[j:]
sub(r'AF_UNIX socketpair \(`tools/rxq_bench.c`, `profiles/r01_rxq_bench.jsonl`\): 1500-B payloads\n  [0-9.]+ M frames/s at batch 64 \(was 1\.44 with one buffer and a blocking check\) and\n  [0-9.]+ M/s \([0-9]+ Gbit/s\) at batch 512 \(was 2\.47\); 64-B payloads [0-9.]+ M/s at batch 512\n  \(was 2\.74\); the same socket without verification [0-9.]+ M/s \(1500 B\) and [0-9.]+ M/s \(64 B\)\.',
    f"AF_UNIX socketpair (`tools/rxq_bench.c`, `profiles/r01_rxq_bench.jsonl`): 1500-B payloads\n  {r(1,1500,64)['Mframes_s']:.2f} M frames/s at batch 64 (was 1.44 with one buffer and a blocking check) and\n  {r(1,1500,512)['Mframes_s']:.2f} M/s ({r(1,1500,512)['Gbit_s']:.0f} Gbit/s) at batch 512 (was 2.47); 64-B payloads {r(1,64,512)['Mframes_s']:.2f} M/s at batch 512\n  (was 2.74); the same socket without verification {r(0,1500,64)['Mframes_s']:.2f} M/s (1500 B) and {r(0,64,512)['Mframes_s']:.2f} M/s (64 B).")
open(p,'w').write(s)
print('ok')
