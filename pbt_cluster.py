"""Reference-compatible module (reference ``pbt_cluster.py``): the PBT master."""
from distributedtf_amd.pbt.cluster import PBTCluster, SPMDPopulation, copy_member_files  # noqa: F401
