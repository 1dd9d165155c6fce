"""The hand-written device scan / sort of lumo_amd/csrc/device/scan.h has no CPU build; these
checks cover its host-visible contract: the header is free of library primitives (no hipCUB left in
the device code), and the library no longer links rocPRIM's sort kernels."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = os.path.join(ROOT, "lumo_amd", "csrc", "device")


def test_no_library_scan_or_sort_in_device_code():
    for f in os.listdir(DEV):
        text = open(os.path.join(DEV, f)).read()
        assert not re.search(r"hipcub|rocprim|cub::", text), f
