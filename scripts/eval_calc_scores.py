"""Drop-in for the reference's scripts/eval_calc_scores.py: same command line, same output
files (bop_toolkit_amd.eval_calc_scores)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bop_toolkit_amd.eval_calc_scores import main  # noqa: E402

if __name__ == "__main__":
  main()
