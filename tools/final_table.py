#!/usr/bin/env python3
"""Markdown rows of DESIGN.md's "every BASELINE config" table from one
session's bench lines (profiles/<round>/bench/<session>_<step>.json).

    python tools/final_table.py r04z3 [--round r04]
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = [  # (step(s), config, workload, round-3 final FPS)
    (("drv", "drv2"), "headline, the driver's command (`--steps 20 --warmup 5`)", "knot stand-in 1920×1080",
     "driver r03: 8,662"),
    (("knot",), "headline, 1,000 frames", "knot stand-in 1920×1080", "10,286-10,312"),
    (("knot_lanes",), "headline, 1,000 frames, two lanes (`--inflight 2`)", "knot stand-in 1920×1080", "10,286-10,312"),
    (("dragon",), "C4 (N=1)", "dragon stand-in 1920×1080", "16,460-16,543"),
    (("dragon960",), "C3", "dragon stand-in 960×540", "46,568-46,768"),
    (("knot960",), "—", "knot stand-in 960×540", "30,569-30,692"),
    (("c2",), "C2", "rabbit_70k 960×540, flat list", "67.9; 71.6-71.7"),
    (("c5",), "C5 (N=1)", "happy stand-in 3840×2160 + shadow ray per hit", "2,638-2,650"),
    (("fill",), "fill", "dragon 1920×1080, 93.4 % coverage", "1,347-1,351"),
    (("fill960",), "fill", "dragon 960×540", "5,068-5,087"),
    (("fillrabbit",), "fill", "rabbit_70k 1920×1080, 94.6 %", "1,734-1,747"),
    (("dragon_shadow",), "—", "dragon 1080p + shadow ray per hit", "5,032-5,044"),
    (("knot_shadow",), "—", "knot 1080p + shadow ray per hit", "4,559-4,564"),
    (("big",), "—", "3.1M-triangle stand-in 1080p", "12,961-12,968"),
    (("anim", "anim2", "anim3"), "—", "dragon 1080p, key sequence `R+W.Q.T.W`, three runs", "11,441-12,496"),
    (("anim10k",), "—", "the same, 10,000 frames (the object behind the eye from tick ~1,000)", "11,290-11,360"),
    (("rehearse",), "—", "knot 1080p through the N > 1 loop at one rank (`--rehearse-gather`)", "10,163-10,282"),
    (("c1",), "C1", "tester 320×180, CPU path (oracle, 16 threads)", "558-571"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("--round", default="r04")
    a = ap.parse_args()
    d = os.path.join(ROOT, "profiles", a.round, "bench")
    print("| config | workload | FPS (round 3 final) | loop | kernel | frac (bound) |")
    print("|---|---|---|---|---|---|")
    for steps, cfg, wl, r3 in ROWS:
        lines = []
        for s in steps:
            p = os.path.join(d, f"{a.session}_{s}.json")
            if os.path.exists(p):
                lines.append(json.load(open(p)))
        if not lines:
            continue
        fps = " / ".join(f"{x['value']:,.0f}" if x["value"] >= 100 else f"{x['value']:.1f}" for x in lines)
        x = lines[0]
        rf = x.get("roofline") or {}
        host = x.get("host") or {}
        fl = host.get("frames_in_flight")
        loop = ("multi-frame" + (f", {rf.get('kernel_options', {}).get('rays_per_wave')} rays"
                                 if rf.get("kernel_options", {}).get("rays_per_wave") != 16 else "")
                if fl == "multi-frame launches" else ("lanes" + (" + gather" if s == "rehearse" else "")) if fl else "—")
        ks = [1e3 * y["roofline"]["kernel_ms_avg"] for y in lines if y.get("roofline")]
        if ks:
            kern = (f"{min(ks):.1f}-{max(ks):.1f} µs" if max(ks) - min(ks) >= 0.1 else f"{ks[0]:.1f} µs")
            if min(ks) > 1000:
                kern = f"{min(ks) / 1e3:.2f} ms"
        else:
            kern = "—"
        frac = (f"{rf['frac']:.3f} ({rf.get('bound', '').upper() if rf.get('bound') == 'hbm' else 'VALU'})"
                if rf.get("frac") is not None else "—")
        if rf.get("unit") == "TFLOP/s":
            frac = f"{rf['frac']:.3f} of {rf['peak']} TFLOP/s"
        if s in ("rehearse",):
            kern, frac = "—", "—"
        print(f"| {cfg} | {wl} | {fps} ({r3}) | {loop} | {kern} | {frac} |")


if __name__ == "__main__":
    main()
