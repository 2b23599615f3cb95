"""Spark SQL types: pyspark's when it is importable, else a minimal stand-in with the same
``names`` / ``fieldNames()`` / ``simpleString()`` behaviour so the schema contract
(reference test_segment.py:50-56, test_pixel.py:8-14, test_chip.py:8-14) holds without a JVM."""
try:  # pragma: no cover - pyspark is not installed in this image
    from pyspark.sql.types import (ArrayType, ByteType, FloatType, IntegerType, StringType,
                                   StructField, StructType, TimestampType)
    HAVE_PYSPARK = True
except Exception:
    HAVE_PYSPARK = False

    class _Atomic(object):
        _name = None

        def simpleString(self):
            return self._name

        def __eq__(self, other):
            return type(self) is type(other)

        def __hash__(self):
            return hash(self._name)

        def __repr__(self):
            return type(self).__name__ + '()'

    class IntegerType(_Atomic):
        _name = 'int'

    class StringType(_Atomic):
        _name = 'string'

    class FloatType(_Atomic):
        _name = 'float'

    class ByteType(_Atomic):
        _name = 'tinyint'

    class TimestampType(_Atomic):
        _name = 'timestamp'

    class ArrayType(object):
        def __init__(self, elementType, containsNull=True):
            self.elementType = elementType
            self.containsNull = containsNull

        def simpleString(self):
            return 'array<%s>' % self.elementType.simpleString()

        def __eq__(self, other):
            return isinstance(other, ArrayType) and self.elementType == other.elementType

    class StructField(object):
        def __init__(self, name, dataType, nullable=True):
            self.name = name
            self.dataType = dataType
            self.nullable = nullable

        def simpleString(self):
            return '%s:%s' % (self.name, self.dataType.simpleString())

    class StructType(object):
        def __init__(self, fields=None):
            self.fields = list(fields or [])
            self.names = [f.name for f in self.fields]

        def fieldNames(self):
            return list(self.names)

        def simpleString(self):
            return 'struct<%s>' % ','.join(f.simpleString() for f in self.fields)

        def __iter__(self):
            return iter(self.fields)

        def __len__(self):
            return len(self.fields)


def require_pyspark(what):
    if not HAVE_PYSPARK:
        raise ImportError('%s needs pyspark, which is not installed' % what)
