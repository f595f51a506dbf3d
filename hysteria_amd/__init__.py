"""hysteria_amd -- Hysteria's Salamander packet obfuscation (extras/obfs) on AMD MI355X.

The product is ``libhyobfs.so`` (gfx950 HIP kernels behind the C ABI of
``include/hyobfs.h``); this package is its Python host binding.
"""
from . import gecko  # noqa: F401
from .conn import SalamanderPacketConn, wrap_packet_conn_salamander  # noqa: F401
from .gecko import GeckoOptions, GeckoPacketConn, wrap_packet_conn_gecko  # noqa: F401
from .salamander import (  # noqa: F401
    SM_KEY_LEN,
    SM_PSK_MIN_LEN,
    SM_SALT_LEN,
    UDP_BUFFER_SIZE,
    PSKTooShortError,
    SalamanderObfuscator,
    build_id,
    deobfuscate_batch_sharded,
    device_count,
    device_pci_bus_id,
    new_salamander_obfuscator,
    obfuscate_batch_sharded,
    synth_bimodal_lengths,
    synth_stream,
    synth_u64,
    workspace_size,
)

__all__ = [
    "SM_KEY_LEN", "SM_PSK_MIN_LEN", "SM_SALT_LEN", "UDP_BUFFER_SIZE", "PSKTooShortError",
    "SalamanderObfuscator", "device_count", "device_pci_bus_id", "new_salamander_obfuscator", "synth_bimodal_lengths",
    "synth_stream", "synth_u64", "workspace_size", "SalamanderPacketConn", "wrap_packet_conn_salamander",
    "obfuscate_batch_sharded", "deobfuscate_batch_sharded", "gecko", "GeckoOptions", "GeckoPacketConn",
    "wrap_packet_conn_gecko", "build_id",
]
