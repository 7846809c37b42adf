from .aggregator import Aggregator
from .sail_recon import SailRecon
