# frozen_string_literal: true

# Redis::BloomfilterDriver::HipLua — the Lua driver's scalable filter on the device
# (`driver: 'hip-lua'`).  Same Redis layout as lib/bloomfilter_driver/lua.rb and
# vendor/assets/lua/add.lua / check.lua, so the two drivers read each other's filters:
#   KEYS[1]:count  items that set a new bit (add.lua:5-11, 48-50)
#   KEYS[1]:n      layer n's bitstring, SETBIT layout (add.lua:17, 38)
# The layers live in HBM behind the bf_lua_* entry points of include/bfhip.h.
# Attaching (`redis=`) loads the count and every layer; sync: :write_through (default)
# writes the layers an insert touched back with SETRANGE and the count with SET, then
# EXPIREs those layers when an expire is given (add.lua:51-53); sync: :manual waits
# for #flush.
require_relative 'hip'

class Redis
  module BloomfilterDriver
    # FFI binding of the bf_lua_* block of include/bfhip.h.
    module HipLuaFFI
      extend FFI::Library
      ffi_lib ENV.fetch('BFHIP_LIB', File.expand_path('../../../lib/libbfhip.so', __dir__))

      attach_function :bf_lua_create, %i[double double pointer pointer], :int, blocking: true
      attach_function :bf_lua_destroy, [:pointer], :int, blocking: true
      attach_function :bf_lua_last_error, [:pointer], :string
      attach_function :bf_lua_insert_many, %i[pointer pointer pointer uint64 pointer pointer], :int, blocking: true
      attach_function :bf_lua_insert_many_changes,
                      %i[pointer pointer pointer uint64 pointer pointer pointer uint64 pointer], :int, blocking: true
      attach_function :bf_lua_include_many, %i[pointer pointer pointer uint64 pointer], :int, blocking: true
      attach_function :bf_lua_clear, [:pointer], :int, blocking: true
      attach_function :bf_lua_get_count, %i[pointer pointer], :int
      attach_function :bf_lua_set_count, %i[pointer uint64], :int
      attach_function :bf_lua_layers, %i[pointer pointer], :int
      attach_function :bf_lua_export_layer, %i[pointer uint32 pointer uint64 pointer], :int, blocking: true
      attach_function :bf_lua_import_layer, %i[pointer uint32 pointer uint64], :int, blocking: true
      attach_function :bf_lua_index, %i[double uint64 pointer], :int
    end

    class HipLua
      attr_reader :redis

      CHANGES_MAX_KEYS = 64   # batches up to this many keys sync by SETBIT replay
      LAYER_SHIFT = 58        # BF_LUA_LAYER_SHIFT

      def initialize(options = {})
        @options = options
        @sync = (options[:sync] || :write_through).to_sym
        raise ArgumentError, 'sync must be :write_through or :manual' unless %i[write_through manual].include?(@sync)

        # ARGV[1], ARGV[2] reach Lua as strings and are read back as numbers (add.lua:1-2)
        @entries = options[:size].to_f
        @precision = options[:error_rate].to_f
        cfg = HipFFI::Config.new
        cfg[:struct_size] = HipFFI::Config.size
        cfg[:device] = options.fetch(:device, -1)
        out = FFI::MemoryPointer.new(:pointer)
        check(HipLuaFFI.bf_lua_create(@entries, @precision, cfg, out), nil)
        @handle = FFI::AutoPointer.new(out.read_pointer, HipLuaFFI.method(:bf_lua_destroy))
        @deadlines = {}   # layer => monotonic deadline of its mirrored TTL (add.lua:51-53)
      end

      def redis=(redis)
        @redis = redis
        reload if redis
      end

      # lua.rb:19-21 (add.lua), one EVALSHA per key in order; returns each key's INCR flag.
      def insert(data, expire = nil)
        insert_many([data], expire).first
      end

      def insert_many(keys, expire = nil)
        expire_if_due
        buf, offs, n = HipFFI.pack(keys)
        flags = FFI::MemoryPointer.new(:uint8, [n, 1].max)
        mask = FFI::MemoryPointer.new(:uint64)
        if @redis && @sync == :write_through && n <= CHANGES_MAX_KEYS
          # per-key inserts replay the SETBITs that changed a layer (add.lua:43-47), not whole layers
          cap = [64 * n, 1].max
          out = FFI::MemoryPointer.new(:uint64, cap)
          cnt = FFI::MemoryPointer.new(:uint64)
          check(HipLuaFFI.bf_lua_insert_many_changes(@handle, buf, offs, n, flags, mask, out, cap, cnt))
          touched = (0...64).select { |i| mask.read_uint64[i] == 1 }.map { |i| i + 1 }
          flips = out.read_array_of_uint64(cnt.read_uint64)
          @redis.pipelined do
            flips.each { |f| @redis.setbit(layer_key(f >> LAYER_SHIFT), f & ((1 << LAYER_SHIFT) - 1), 1) }
            @redis.set("#{@options[:key_name]}:count", device_count.to_s) unless touched.empty?
          end
        else
          check(HipLuaFFI.bf_lua_insert_many(@handle, buf, offs, n, flags, mask))
          touched = (0...64).select { |i| mask.read_uint64[i] == 1 }.map { |i| i + 1 }
          write(touched) if !touched.empty? && @redis && @sync == :write_through
        end
        if !touched.empty? && expire
          t0 = now   # before EXPIRE: never after the server's deadline
          touched.each do |l|
            @deadlines[l] = t0 + expire
            @redis.expire(layer_key(l), expire) if @redis && @sync == :write_through
          end
        end
        flags.read_array_of_uint8(n).map { |b| b == 1 }
      end

      # lua.rb:23-26 (check.lua)
      def include?(key)
        include_many?([key]).first
      end

      def include_many?(keys)
        expire_if_due
        buf, offs, n = HipFFI.pack(keys)
        out = FFI::MemoryPointer.new(:uint8, [n, 1].max)
        check(HipLuaFFI.bf_lua_include_many(@handle, buf, offs, n, out))
        out.read_array_of_uint8(n).map { |b| b == 1 }
      end

      # lua.rb:28-30
      def clear
        check(HipLuaFFI.bf_lua_clear(@handle))
        @deadlines.clear
        @redis&.keys("#{@options[:key_name]}:*")&.each { |k| @redis.del(k) }
      end

      # Every layer and the count -> Redis.
      def flush
        write((1..layers).to_a) if @redis
      end

      # Redis -> device layers and count (replace).
      def reload
        check(HipLuaFFI.bf_lua_clear(@handle))
        @deadlines.clear
        count = @redis.get("#{@options[:key_name]}:count").to_i
        check(HipLuaFFI.bf_lua_set_count(@handle, count))
        return if count.zero?

        idx = FFI::MemoryPointer.new(:uint32)
        check(HipLuaFFI.bf_lua_index(@entries, count, idx))
        (1..idx.read_uint32).each do |l|
          t0 = now
          pttl = @redis.pttl(layer_key(l))
          str = @redis.get(layer_key(l))
          next if str.nil? || str.empty?

          mem = FFI::MemoryPointer.new(:uint8, str.bytesize)
          mem.put_bytes(0, str)
          check(HipLuaFFI.bf_lua_import_layer(@handle, l, mem, str.bytesize))
          @deadlines[l] = t0 + pttl / 1000.0 if pttl.positive?
        end
      end

      private

      # Layers whose mirrored TTL passed are gone in Redis: empty them on the device too
      # (the count key has no TTL and stays, as in Redis).
      def expire_if_due
        t = now
        @deadlines.select { |_, d| t >= d }.each_key do |l|
          @deadlines.delete(l)
          check(HipLuaFFI.bf_lua_import_layer(@handle, l, nil, 0))
          @redis.del(layer_key(l)) if @redis && @sync == :write_through
        end
      end

      def now
        Process.clock_gettime(Process::CLOCK_MONOTONIC)
      end

      def layer_key(layer)
        "#{@options[:key_name]}:#{layer}"
      end

      def layers
        n = FFI::MemoryPointer.new(:uint32)
        check(HipLuaFFI.bf_lua_layers(@handle, n))
        n.read_uint32
      end

      def write(layer_list)
        layer_list.each do |l|
          len = FFI::MemoryPointer.new(:uint64)
          check(HipLuaFFI.bf_lua_export_layer(@handle, l, nil, 0, len))
          n = len.read_uint64
          next if n.zero?

          buf = FFI::MemoryPointer.new(:uint8, n)
          check(HipLuaFFI.bf_lua_export_layer(@handle, l, buf, n, len))
          @redis.setrange(layer_key(l), 0, buf.read_bytes(n))
        end
        @redis.set("#{@options[:key_name]}:count", device_count.to_s)
      end

      def device_count
        count = FFI::MemoryPointer.new(:uint64)
        check(HipLuaFFI.bf_lua_get_count(@handle, count))
        count.read_uint64
      end

      def check(rc, handle = @handle)
        return if rc == HipFFI::BF_OK

        msg = HipLuaFFI.bf_lua_last_error(handle)
        raise ArgumentError, msg if [HipFFI::BF_EINVAL, HipFFI::BF_ERANGE].include?(rc)

        raise "bfhip error #{rc}: #{msg}"
      end
    end
  end
end
