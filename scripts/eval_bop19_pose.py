"""Drop-in for the reference's scripts/eval_bop19_pose.py: same command line, same output
files (bop_toolkit_amd.eval_bop19_pose)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bop_toolkit_amd.eval_bop19_pose import main  # noqa: E402

if __name__ == "__main__":
  main()
