"""Summarise tools/pmc_learner.sh's counter dump (``NAME value`` lines) into
the derived shares recorded in profiles/r*_learner_pmc.txt."""
import sys

vals = {}
for line in open(sys.argv[1]):
    parts = line.split()
    if len(parts) == 2 and parts[0].startswith("SQ_"):
        try:
            vals[parts[0]] = float(parts[1])
        except ValueError:
            pass
for k in sorted(vals):
    print(k, int(vals[k]))
print()
wc = vals["SQ_WAVE_CYCLES"]


def line(label, expr, x):
    print(f"{label:<30}{expr:<40}= {x:.3f}")


line("waiting share of wave cycles", "SQ_WAIT_ANY / SQ_WAVE_CYCLES", vals["SQ_WAIT_ANY"] / wc)
line("issuing share of wave cycles", "SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES", vals["SQ_ACTIVE_INST_ANY"] / wc)
line("VALU-active share", "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES", vals["SQ_ACTIVE_INST_VALU"] / wc)
line("LDS-active share", "SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES", vals["SQ_ACTIVE_INST_LDS"] / wc)
line("LDS bank-conflict share", "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE", vals["SQ_LDS_BANK_CONFLICT"] / vals["SQ_LDS_IDX_ACTIVE"])
print(f"VALU instructions per MFMA    {vals['SQ_INSTS_VALU'] / vals['SQ_INSTS_MFMA']:.1f} "
      f"(VALU {int(vals['SQ_INSTS_VALU'])}, MFMA {int(vals['SQ_INSTS_MFMA'])}, LDS {int(vals['SQ_INSTS_LDS'])}, "
      f"SALU {int(vals['SQ_INSTS_SALU'])})")
