"""ccdc.chip -- per-chip dates projection (mirror of reference ccdc/chip.py)."""
from ccdc._types import ArrayType, IntegerType, StringType, StructField, StructType, require_pyspark


def table():
    """Cassandra table name"""
    return 'chip'


def schema():
    """ Schema for chip dataframe """
    return StructType([
        StructField('cx', IntegerType(), nullable=False),
        StructField('cy', IntegerType(), nullable=False),
        StructField('dates', ArrayType(StringType()), nullable=False),
    ])


def dataframe(ctx, ccd):
    return ccd.select(schema().fieldNames())


def read(ctx, ids):
    require_pyspark('ccdc.chip.read (Cassandra storage is out of scope)')


def write(ctx, df):
    require_pyspark('ccdc.chip.write (Cassandra storage is out of scope)')
