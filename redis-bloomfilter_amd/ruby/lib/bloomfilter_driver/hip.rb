# frozen_string_literal: true

# Redis::BloomfilterDriver::Hip — the MI355X driver for the redis-bloomfilter gem.
#
# Drop-in next to lib/bloomfilter_driver/ruby.rb and lua.rb: the facade
# resolves `driver: 'hip'` to this class through `const_get`
# (lib/redis/bloomfilter.rb:43, driver_name at :77-79), passes the whole
# options hash (with :bits and :hashes, :25-28) and then sets `redis=` (:45).
#
# The filter lives in HBM behind libbfhip.so (include/bfhip.h); Ruby talks to
# it through FFI with `blocking: true`, so the GVL is released during device
# work.  Redis keeps the same bitstring the ruby driver writes (SETBIT layout,
# MSB-first), so the two drivers read each other's filters:
#   * attaching (`redis=`) imports an existing key and its TTL;
#   * sync: :write_through (default) writes back, with one SETRANGE per range,
#     the 64 KiB blocks of the string an insert changed (the device's dirty-block
#     map, bf_track_dirty; SETRANGE keeps the TTL and grows the string exactly
#     like SETBIT), then EXPIREs iff a bit flipped and an expire was given
#     (ruby.rb:61-62);
#   * sync: :manual leaves Redis alone until #flush (changes since the last one).
# Every write is cut into SETRANGE calls of at most :chunk_bytes (default 8 MiB)
# and a longer key is read back with GETRANGE chunks, so multi-GB filters move
# through a server whose proto-max-bulk-len admits them (SURVEY §8 f2).
# Extra options: :device (HIP ordinal), :devices (ordinals or a count) + :mode (:replicated or
# :partitioned) for one filter over several GPUs, :sync, :batch_keys, :batch_bytes, :chunk_bytes.
require 'ffi'

class Redis
  module BloomfilterDriver
    # FFI binding of include/bfhip.h (host-pointer entry points only).
    module HipFFI
      extend FFI::Library
      ffi_lib ENV.fetch('BFHIP_LIB', File.expand_path('../../../lib/libbfhip.so', __dir__))

      BF_OK = 0
      BF_EINVAL = 1
      BF_ERANGE = 5
      BF_IMPORT_REPLACE = 0
      BF_FLAG_ENGINE_MD5 = 2
      BF_FLAG_ENGINE_SHA1 = 4

      # `data.to_s` bytes (ruby.rb:42) of every key, packed as (bytes, uint64 offsets[n+1], n).
      def self.pack(keys)
        strs = keys.map { |k| k.to_s.b }
        n = strs.size
        buf = FFI::MemoryPointer.new(:uint8, [strs.sum(&:bytesize), 1].max)
        offs = FFI::MemoryPointer.new(:uint64, n + 1)
        pos = 0
        offsets = [0]
        strs.each do |s|
          buf.put_bytes(pos, s) unless s.empty?
          pos += s.bytesize
          offsets << pos
        end
        offs.write_array_of_uint64(offsets)
        [buf, offs, n]
      end

      BF_MAX_DEVICES = 16
      BF_MODE_REPLICATED = 0
      BF_MODE_PARTITIONED = 1

      # struct bf_config (include/bfhip.h)
      class Config < FFI::Struct
        layout :struct_size, :uint32, :device, :int32, :batch_keys, :uint64, :batch_bytes, :uint64,
               :shard_count, :uint32, :shard_index, :uint32, :shard_block_log2, :uint32, :flags, :uint32,
               :device_count, :uint32, :mode, :uint32, :devices, [:int32, BF_MAX_DEVICES]
      end

      attach_function :bf_version, [], :string
      attach_function :bf_last_error, [:pointer], :string
      attach_function :bf_create, %i[uint64 uint32 pointer pointer], :int, blocking: true
      attach_function :bf_destroy, [:pointer], :int, blocking: true
      attach_function :bf_insert_many, %i[pointer pointer pointer uint64 pointer pointer], :int, blocking: true
      attach_function :bf_include_many, %i[pointer pointer pointer uint64 pointer], :int, blocking: true
      attach_function :bf_clear, [:pointer], :int, blocking: true
      attach_function :bf_export_redis, %i[pointer pointer uint64 pointer], :int, blocking: true
      attach_function :bf_import_redis, %i[pointer pointer uint64 uint32], :int, blocking: true
      attach_function :bf_track_dirty, %i[pointer uint32], :int, blocking: true
      attach_function :bf_dirty_ranges, %i[pointer pointer uint32 pointer pointer uint32], :int, blocking: true
      attach_function :bf_export_range, %i[pointer uint64 uint64 pointer], :int, blocking: true
      attach_function :bf_insert_many_changes, %i[pointer pointer pointer uint64 pointer uint64 pointer], :int,
                      blocking: true
      attach_function :bf_indexes, %i[pointer uint64 uint64 uint32 pointer], :int, blocking: true
    end

    class Hip
      attr_reader :redis

      def initialize(options = {})
        @options = options
        bits = options[:bits]
        # ruby.rb:51 would raise ZeroDivisionError on the first insert
        raise ArgumentError, 'filter size in bits must be positive' unless bits.is_a?(Integer) && bits.positive?

        @sync = (options[:sync] || :write_through).to_sym
        raise ArgumentError, 'sync must be :write_through or :manual' unless %i[write_through manual].include?(@sync)

        cfg = HipFFI::Config.new
        cfg[:struct_size] = HipFFI::Config.size
        cfg[:device] = options.fetch(:device, -1)
        cfg[:batch_keys] = options.fetch(:batch_keys, 0)
        cfg[:batch_bytes] = options.fetch(:batch_bytes, 0)
        cfg[:flags] = config_flags
        configure_devices(cfg, options)
        out = FFI::MemoryPointer.new(:pointer)
        check(HipFFI.bf_create(bits, options[:hashes], cfg, out), nil)
        @handle = FFI::AutoPointer.new(out.read_pointer, HipFFI.method(:bf_destroy))
        check(HipFFI.bf_track_dirty(@handle, 1))
        @chunk = options.fetch(:chunk_bytes, 8 << 20)
        raise ArgumentError, 'chunk_bytes must be positive' unless @chunk.positive?
        @deadline = nil
      end

      # attr_accessor :redis (ruby.rb:9); attaching loads the existing filter.
      def redis=(redis)
        @redis = redis
        reload if redis
      end

      # ruby.rb:15-17
      def insert(data, expire = nil)
        insert_many([data], expire)
      end

      # Batched insert; returns true iff some bit flipped (the ruby driver's !found).
      def insert_many(keys, expire = nil)
        expire_if_due
        buf, offs, n = pack(keys)
        changed = insert_setbits(buf, offs, n) if @redis && @sync == :write_through && changes_path?(n)
        if changed.nil?
          flag = FFI::MemoryPointer.new(:uint8)
          check(HipFFI.bf_insert_many(@handle, buf, offs, n, flag, nil))
          changed = flag.read_uint8 == 1
          flush if changed && @redis && @sync == :write_through
        end
        if changed
          if expire
            @deadline = now + expire   # taken before EXPIRE: never after the server's deadline
            @redis.expire(@options[:key_name], expire) if @redis && @sync == :write_through
          end
        end
        changed
      end

      # ruby.rb:20-30
      def include?(key)
        include_many?([key]).first
      end

      def include_many?(keys)
        expire_if_due
        buf, offs, n = pack(keys)
        out = FFI::MemoryPointer.new(:uint8, [n, 1].max)
        check(HipFFI.bf_include_many(@handle, buf, offs, n, out))
        out.read_array_of_uint8(n).map { |b| b == 1 }
      end

      # ruby.rb:33-35
      def clear
        check(HipFFI.bf_clear(@handle))
        @deadline = nil
        @redis&.del(@options[:key_name])
      end

      # Device changes -> Redis, one SETRANGE per dirty range (keeps the TTL, grows
      # like SETBIT); full: true sends the whole string.  Returns the bytes sent.
      def flush(full: false)
        ranges = dirty_ranges(clear: !@redis.nil?)
        return 0 unless @redis

        if full
          n = export_len
          ranges = n.positive? ? [[0, n]] : []
        end
        ranges.sum do |off, len|
          (off...(off + len)).step(@chunk).sum do |c|
            n = [@chunk, off + len - c].min
            buf = FFI::MemoryPointer.new(:uint8, n)
            check(HipFFI.bf_export_range(@handle, c, n, buf))
            @redis.setrange(@options[:key_name], c, buf.read_bytes(n))
            n
          end
        end
      end

      # [[byte offset, length], ...] changed since the last clear (bf_dirty_ranges).
      def dirty_ranges(clear: true)
        n = FFI::MemoryPointer.new(:uint32)
        loop do
          check(HipFFI.bf_dirty_ranges(@handle, nil, 0, n, nil, 0))
          cap = [n.read_uint32, 1].max
          out = FFI::MemoryPointer.new(:uint64, 2 * cap)
          rc = HipFFI.bf_dirty_ranges(@handle, out, cap, n, nil, clear ? 1 : 0)
          next if rc == HipFFI::BF_ERANGE && n.read_uint32 > cap   # grew meanwhile

          check(rc)
          return out.read_array_of_uint64(2 * n.read_uint32).each_slice(2).to_a
        end
      end

      # Redis -> device filter (replace).
      def reload
        str = read_key
        @deadline = nil
        if str.nil?
          check(HipFFI.bf_clear(@handle))
          return
        end
        mem = FFI::MemoryPointer.new(:uint8, [str.bytesize, 1].max)
        mem.put_bytes(0, str)
        check(HipFFI.bf_import_redis(@handle, mem, str.bytesize, HipFFI::BF_IMPORT_REPLACE))
        dirty_ranges(clear: true)   # device == Redis now
        t0 = now
        pttl = @redis.pttl(@options[:key_name])   # milliseconds: no whole-second rounding
        @deadline = t0 + pttl / 1000.0 if pttl.positive?
      end

      # The Redis string of the device filter (GET key_name after the same SETBITs).
      def export
        n = export_len
        buf = FFI::MemoryPointer.new(:uint8, [n, 1].max)
        len = FFI::MemoryPointer.new(:uint64)
        check(HipFFI.bf_export_redis(@handle, buf, n, len))
        buf.read_bytes(len.read_uint64)
      end

      protected

      # Ruby#indexes_for (ruby.rb:41-55): the k offsets of one key, from the device kernel.
      def indexes_for(data)
        s = data.to_s.b
        key = FFI::MemoryPointer.new(:uint8, [s.bytesize, 1].max)
        key.put_bytes(0, s)
        out = FFI::MemoryPointer.new(:uint64, @options[:hashes])
        check(HipFFI.bf_indexes(key, s.bytesize, @options[:bits], @options[:hashes], out), nil)
        out.read_array_of_uint64(@options[:hashes])
      end

      # bf_config.flags of the device filter (HipTest picks a hash engine here).
      def config_flags
        0
      end

      # bf_insert_many_changes limits (include/bfhip.h)
      CHANGES_MAX_PROBES = 4096
      CHANGES_MAX_BYTES = 64 << 10
      BF_DIRTY_BLOCK_BYTES = 65_536

      # Write-through replays the SETBITs an insert flipped (pipelined like ruby.rb:58-60) instead
      # of SETRANGEing whole 64 KiB blocks while that costs Redis less: a pipelined SETBIT is about
      # as much server work as ~1 KB of SETRANGE (SETBIT_BYTES), so per-key calls always, and
      # batches while their probes stay under 1/1024 of the bytes the block flush would send.  A
      # concurrent writer's bits in those blocks are never overwritten either.
      SETBIT_BYTES = 1024

      def changes_path?(n)
        return false unless @options[:devices].nil?

        probes = n * @options[:hashes]
        return true if probes <= CHANGES_MAX_PROBES

        reach = [@options[:bits], @options[:hashes] * 0xFFFFFFFF + 1].min
        blocks = ((reach + 7) / 8 + BF_DIRTY_BLOCK_BYTES - 1) / BF_DIRTY_BLOCK_BYTES
        probes * SETBIT_BYTES <= [probes, blocks].min * BF_DIRTY_BLOCK_BYTES
      end

      # bf_insert_many_changes in pieces of <= CHANGES_MAX_PROBES probes and CHANGES_MAX_BYTES
      # key bytes; nil (nothing inserted) when one key alone is longer than a piece may be.
      def insert_setbits(buf, offs, n)
        o = offs.read_array_of_uint64(n + 1)
        return nil if (0...n).any? { |j| o[j + 1] - o[j] > CHANGES_MAX_BYTES }

        per = [CHANGES_MAX_PROBES / @options[:hashes], 1].max
        flips = []
        i = 0
        while i < n
          j = [i + per, n].min
          j -= 1 while o[j] - o[i] > CHANGES_MAX_BYTES
          cap = (j - i) * @options[:hashes]
          out = FFI::MemoryPointer.new(:uint64, [cap, 1].max)
          cnt = FFI::MemoryPointer.new(:uint64)
          check(HipFFI.bf_insert_many_changes(@handle, buf, offs + 8 * i, j - i, out, cap, cnt))
          flips.concat(out.read_array_of_uint64(cnt.read_uint64))
          i = j
        end
        unless flips.empty?
          name = @options[:key_name]
          @redis.pipelined { flips.each { |b| @redis.setbit(name, b, 1) } }
        end
        !flips.empty?
      end

      # `devices: [0, 1, ...]` (or a count) and `mode: :replicated | :partitioned`: one filter
      # over several GPUs from this process (bf_config.device_count / devices / mode).
      def configure_devices(cfg, options)
        devices = options[:devices]
        return if devices.nil?

        devices = (0...devices).to_a if devices.is_a?(Integer)
        unless devices.is_a?(Array) && !devices.empty? && devices.size <= HipFFI::BF_MAX_DEVICES
          raise ArgumentError, "devices must list 1..#{HipFFI::BF_MAX_DEVICES} GPU ordinals"
        end

        mode = (options[:mode] || :replicated).to_sym
        raise ArgumentError, 'mode must be :replicated or :partitioned' unless %i[replicated partitioned].include?(mode)

        cfg[:device_count] = devices.size
        cfg[:mode] = mode == :partitioned ? HipFFI::BF_MODE_PARTITIONED : HipFFI::BF_MODE_REPLICATED
        devices.each_with_index { |d, i| cfg[:devices][i] = d }
      end

      private

      def export_len
        len = FFI::MemoryPointer.new(:uint64)
        check(HipFFI.bf_export_redis(@handle, nil, 0, len))
        len.read_uint64
      end

      # GET, or GETRANGE chunks for a key longer than :chunk_bytes.
      def read_key
        key = @options[:key_name]
        n = @redis.strlen(key)
        return @redis.get(key) if n <= @chunk

        (0...n).step(@chunk).map { |c| @redis.getrange(key, c, [c + @chunk, n].min - 1) }.join.b
      end

      # `data.to_s` bytes (ruby.rb:42), packed as (bytes, uint64 offsets[n+1]).
      def pack(keys)
        HipFFI.pack(keys)
      end

      # The mirrored TTL passed: drop the device copy and (write-through) the key, so device
      # and Redis agree from here on (the key was due to vanish within a round trip anyway).
      def expire_if_due
        return unless @deadline && now >= @deadline

        @deadline = nil
        check(HipFFI.bf_clear(@handle))
        @redis.del(@options[:key_name]) if @redis && @sync == :write_through
      end

      def now
        Process.clock_gettime(Process::CLOCK_MONOTONIC)
      end

      def check(rc, handle = @handle)
        return if rc == HipFFI::BF_OK

        msg = HipFFI.bf_last_error(handle)
        raise ArgumentError, msg if [HipFFI::BF_EINVAL, HipFFI::BF_ERANGE].include?(rc)

        raise "bfhip error #{rc}: #{msg}"
      end
    end
  end
end
