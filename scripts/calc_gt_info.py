"""Drop-in for the reference's scripts/calc_gt_info.py (bop_toolkit_amd.gt_side info)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bop_toolkit_amd.gt_side import main  # noqa: E402

if __name__ == "__main__":
  main(["info"] + sys.argv[1:])
