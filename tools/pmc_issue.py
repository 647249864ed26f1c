#!/usr/bin/env python3
"""What binds each list kernel, from the PMC groups of tools/pmc_ab.sh (a tools/pmc_summary.py
text file): per kernel and launch

  valu_busy          VALU issue: SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) over the
                     1024 SIMDs x the launch's quad-cycles (GRBM_GUI_ACTIVE summed over 8 XCDs)
  l1_lookups_per_clk L1 (TCP) tag lookups per clock per CU (one per clock is the ceiling)
  valu_per_wave, vmem_per_wave, tcp_per_vmem, lds_conflict_frac (bank-conflict cycles over the
                     launch's cycles per CU), ta_busy (texture-address unit busy fraction)

usage: python tools/pmc_issue.py gpurun_out/pmc_base.txt case > profiles/pmc_issue.json
"""
import json
import sys

NSIMD, NCU, NXCD = 1024, 256, 8


def parse(path):
    out, cur = {}, None
    for ln in open(path):
        if not ln.startswith(" "):
            cur = ln.strip().split("<")[0].replace("mph::k_", "")
            out[cur] = {}
        elif cur:
            k, v = ln.split()
            out[cur][k] = float(v)
    return out


def main():
    d = parse(sys.argv[1])
    res = {"case": sys.argv[2] if len(sys.argv) > 2 else "d1m", "source": sys.argv[1],
           "note": "VALU busy = SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4); "
                   "L1 lookups per clock per CU = TCP_TOTAL_CACHE_ACCESSES_sum / (256 x GRBM_GUI_ACTIVE/8)"}
    for k, c in d.items():
        g = c.get("GRBM_GUI_ACTIVE")
        if not g:
            continue
        cyc = g / NXCD
        w = c.get("SQ_WAVES", 0) or 1
        res[k] = {
            "valu_busy": round(c.get("SQ_ACTIVE_INST_VALU", 0) / (NSIMD * cyc / 4), 4),
            "l1_lookups_per_clk": round(c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / (NCU * cyc), 4),
            "valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / w, 1),
            "vmem_per_wave": round(c.get("SQ_INSTS_VMEM_RD", 0) / w, 1),
            "tcp_per_vmem": round(c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / max(c.get("SQ_INSTS_VMEM_RD", 0), 1), 2),
            "lds_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / (NCU * cyc), 4),
            # texture-address unit: TA_BUSY_avr (busy cycles averaged over the TA instances) over
            # the launch's cycles
            "ta_busy": round(c.get("TA_BUSY_avr", 0) / cyc, 4),
            "cycles_per_xcd": round(cyc),
        }
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
