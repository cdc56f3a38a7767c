#!/usr/bin/env python
"""Speed-of-light model of one bench step (BASELINE config 2: HSTU d=512,
L=200, 4 blocks x 8 heads, B=128, 1M-item tables, BCE, jagged rows,
dense-parity table AdamW): algorithmic FLOPs of every GEMM-shaped product and
a lower bound on HBM bytes, priced at the MI355X peaks (2.5 PFLOP/s dense
bf16 MFMA, 8 TB/s HBM; MI355X_MICROARCH.md).  Analytical, no GPU: the floor a
step could reach if every kernel ran at its roof and nothing else ran.

    python scripts/step_model.py [--span 14900] [--measured-ms 5.19] > profiles/r3_step_model.txt

Counting rules (stated so they can be checked):
  * GEMM FLOPs = 2 M N K per product; a linear layer's backward = 2x its
    forward (dX and dW).  Rows = the batch's span rows (valid positions),
    the jagged layout's work (the capacity padding is not counted).
  * HSTU attention: causal pairs of each sequence (lengths U{32..201}, the
    synthetic batches), QK^T and PV forward (2 products), S / dP / dV / dK /
    dQ and the dQ / dK/dV kernels' S and dP recomputes backward (7).
  * HBM bytes: every activation tensor written once by its producer and read
    once by each consumer (bf16 2 B per element); embedding rows read once
    per distinct row; optimizer: parameters, moments and gradients read and
    written once per update; the deferred dense-parity catch-up of the 1M-row
    tables every 16 steps amortised per step.
"""
import argparse

PEAK_FLOPS = 2.5e15   # dense bf16 MFMA
PEAK_BW = 8.0e12      # HBM3E


def model(n, B=128, T=201, d=512, H=8, blocks=4, items=1_000_000, users=1_000_000, p_rows=41462,
          mm=32, defer=16):
    comp = []   # (name, flops, bytes)
    K_item, K_user = d + 40, d + 8   # composed operand widths (item rows | mm | 1 | pad ; user rows | 1 | pad)
    # -- dnn GEMMs (forward + dX + dW)
    f = 2 * n * K_item * d + 2 * n * K_user * d + 2 * (2 * n) * K_item * d
    comp.append(('itemdnn / userdnn GEMMs (seq + pos/neg)', 3 * f, 0))
    # -- projected feature tables P = E W (forward; backward dE + dW)
    comp.append(('feature-table projection P = E W', 3 * 2 * p_rows * d * d, 0))
    # -- HSTU projections
    f = blocks * (2 * n * d * 4 * d + 2 * n * d * d)
    comp.append(('HSTU uvqk + output projections', 3 * f, 0))
    # -- HSTU attention
    lens = range(32, T + 1)
    pairs = B * sum(L * (L + 1) / 2 for L in lens) / len(lens)
    comp.append(('HSTU attention (causal pairs, fwd 2 + bwd 7 products)', blocks * 9 * 2 * pairs * d, 0))
    # -- embedding rows (bytes): item rows of seq + pos + neg, user rows, P read once, pos table
    rows = 3 * n + B
    comp.append(('embedding gathers (distinct rows, P once)', 0, rows * d * 2 + p_rows * d * 2 + n * 4 * 40))
    # -- embedding backward: one gradient row read per distinct row + fp32 row written
    comp.append(('embedding backward (gradient rows once)', 0, rows * d * (2 + 4) + p_rows * d * 4))
    # -- activations, forward: operand blocks, dnn outputs, per layer x / LN / uvqk / attn / gate / out
    width_in = (K_item + d + K_user + d + d) + 2 * (K_item + d)      # gather outputs (seq, pos/neg)
    act_fwd = n * width_in * 2 + 3 * n * d * 2 * 2                  # written + read; dnn outputs
    per_layer = n * 2 * (d + d + 4 * d + 4 * d + d + d + d + d)     # x, LN, uvqk (w+r), attn, LN-gate, out, residual
    act_fwd += blocks * per_layer
    comp.append(('activations forward (write + read once)', 0, act_fwd))
    comp.append(('activations backward (~2x forward)', 0, 2 * act_fwd))
    # -- optimizer
    dense = (d * 16 * d + d) + (d * 9 * d + d) + blocks * (d * 4 * d + 4 * d + d * d + d + 4 * d) + mm * d + 4 * d
    comp.append(('dense AdamW (fp32 p, m, v r/w + grad)', 0, dense * 28))
    touched = 3 * n + B
    comp.append(('table AdamW, touched item/user rows (bf16 p, fp32 m, v)', 0, touched * d * 20))
    comp.append(('table AdamW, small tables every step', 0, p_rows * d * 20))
    comp.append((f'table AdamW catch-up of 1M-row tables / {defer}', 0, (items + users) * d * 20 / defer))
    return comp, pairs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--span', type=float, default=14_900, help='span rows per batch (bench pool: 13,670-16,167)')
    ap.add_argument('--measured-ms', type=float, default=5.19, help='profiles/r3_bench_default.json ms_per_step')
    a = ap.parse_args()
    comp, pairs = model(a.span)
    tf = sum(c[1] for c in comp)
    tb = sum(c[2] for c in comp)
    print(f'# step model, BASELINE config 2 (jagged, {a.span:.0f} span rows, {pairs / 128:.0f} causal pairs / sequence)')
    print(f'{"component":58s} {"GFLOP":>9s} {"MB":>9s} {"us @ roof":>10s}')
    for name, f, b in comp:
        us = max(f / PEAK_FLOPS, b / PEAK_BW) * 1e6
        print(f'{name:58s} {f / 1e9:9.1f} {b / 1e6:9.1f} {us:10.1f}')
    t_mfma, t_hbm = tf / PEAK_FLOPS * 1e3, tb / PEAK_BW * 1e3
    print(f'{"total":58s} {tf / 1e9:9.1f} {tb / 1e6:9.1f}')
    print(f'# floor: MFMA {t_mfma:.3f} ms, HBM {t_hbm:.3f} ms; overlapped max {max(t_mfma, t_hbm):.3f} ms, '
          f'serial sum {t_mfma + t_hbm:.3f} ms')
    print(f'# measured {a.measured_ms:.2f} ms/step = {a.measured_ms / (t_mfma + t_hbm):.1f}x (serial) - '
          f'{a.measured_ms / max(t_mfma, t_hbm):.1f}x (overlapped) the floor')


if __name__ == '__main__':
    main()
