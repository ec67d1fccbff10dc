"""python -m sfs2d VCF POPMAP ... (see sfs2d.cli)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))   # twoDSFS_class.py

from sfs2d.cli import main  # noqa: E402

main()
