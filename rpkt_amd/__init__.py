"""rpkt_amd — MI355X-native batch engine for rpkt's Ether -> (VLAN)* -> IPv4 ->
{TCP, UDP} decode-and-verify path.

  rpkt_amd.records   record layout (include/rpkt_gpu.h) as a numpy dtype
  rpkt_amd.views     EtherFrame / VlanFrame / Ipv4 / Udp / Tcp getters over records
  rpkt_amd.engine    device batch API over the C ABI (librpkt_gpu.so, HIP/gfx950)
  rpkt_amd.gen       seeded synthetic frame generator (librpkt_gen.so, host C++)
"""
from . import records, views  # noqa: F401
from .records import REC_DTYPE, REC_BYTES, STATUS, F_IP_SUM, F_L4_SUM, F_FLOW_EV  # noqa: F401

__version__ = "0.1.0"
