"""`python -m fantoch_amd`: the reference's bote binary (fantoch_bote/src/main.rs); see fantoch_amd/cli.py."""
import sys

from .cli import main

sys.exit(main())
